#!/bin/bash
# Full GPU pass: parity suite, the three bench modes (per-round with the CPU
# baseline, RLC, threshold recovery with its CPU baseline), rocprofv3 kernel
# stats of the per-round and recovery benches.  Stops at the first failure.
export TMPDIR=/tmp
TAG=${TAG:-full}
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step pytest
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
step bench-per-round
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
cat $O/bench.json
step bench-rlc
timeout -k 10 600 python bench.py --mode rlc --no-cpu-baseline > $O/bench_rlc.json 2> $O/bench_rlc.err || exit $?
cat $O/bench_rlc.json
step bench-recover
timeout -k 10 600 python bench.py --mode recover > $O/bench_recover.json 2> $O/bench_recover.err || exit $?
cat $O/bench_recover.json
[ -n "$NO_PROF" ] && exit 0
step prof-per-round
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o bench -- python3 bench.py --no-cpu-baseline --steps 2 > $O/prof.out 2>&1 || exit $?
step prof-recover
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_recover -o bench -- python3 bench.py --mode recover --no-cpu-baseline --steps 2 > $O/prof_recover.out 2>&1 || exit $?
find $O/prof $O/prof_recover -name "*kernel_stats*" -exec head -14 {} \;
