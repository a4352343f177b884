#!/bin/bash
# Round-2 measurement session on the shipped build: the metric bench (10M
# chained rounds: per-round, end-to-end, RLC, CPU baseline), on-G1
# (configs[3]) and threshold recovery (configs[4]) benches, then rocprofv3
# kernel statistics of the default bench.  Stops at the first failure.
export TMPDIR=/tmp
TAG=${TAG:-r02u}
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
if [ -n "$TEST" ]; then
step pytest
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
step smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
fi
step bench
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
head -c 700 $O/bench.json; echo
step bench-on-g1
timeout -k 10 300 python -u bench.py --scheme bls-unchained-on-g1 --rounds 1000000 > $O/bench_on_g1.json 2> $O/bench_on_g1.err || exit $?
step bench-recover
timeout -k 10 300 python -u bench.py --mode recover > $O/bench_recover.json 2> $O/bench_recover.err || exit $?
step rocprof
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o bench -- python3 bench.py --no-cpu-baseline --no-e2e --steps 2 > $O/prof.out 2>&1 || exit $?
python3 tools/rocpd_stats.py $(find $O/prof -name "*results.db" | head -1) > $O/kernel_stats.csv
echo done
