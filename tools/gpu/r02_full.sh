#!/bin/bash
# Round-2 full pass: parity suite, the metric bench (10M, per-round + RLC +
# end-to-end, CPU baseline), on-G1 (configs[3]) and recovery (configs[4])
# benches with their C baselines, multi-process bench rehearsal skipped
# (one GPU).  Stops at the first failure.
export TMPDIR=/tmp
TAG=${TAG:-r02f}
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step pytest
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
step bench
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
step bench-on-g1
timeout -k 10 400 python -u bench.py --scheme bls-unchained-on-g1 --rounds 1000000 > $O/bench_on_g1.json 2> $O/bench_on_g1.err || exit $?
step bench-recover
timeout -k 10 400 python -u bench.py --mode recover > $O/bench_recover.json 2> $O/bench_recover.err || exit $?
echo done
