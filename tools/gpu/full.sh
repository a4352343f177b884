#!/bin/bash
# Full GPU pass: parity suite, the bench modes (per-round chained with the CPU
# baseline, RLC, on-G1, threshold recovery), rocprofv3 kernel statistics of
# the per-round / on-G1 / recovery benches (rocpd database -> CSV summary),
# and the two PMC traffic passes.  Stops at the first failure.
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
step bench-on-g1
timeout -k 10 600 python bench.py --scheme bls-unchained-on-g1 > $O/bench_on_g1.json 2> $O/bench_on_g1.err || exit $?
step bench-recover
timeout -k 10 600 python bench.py --mode recover > $O/bench_recover.json 2> $O/bench_recover.err || exit $?
[ -n "$NO_PROF" ] && exit 0
prof() {  # name, bench args
  step prof-$1
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_$1 -o bench -- python3 bench.py --no-cpu-baseline --steps 2 $2 > $O/prof_$1.out 2>&1 || return $?
  python3 tools/rocpd_stats.py $(find $O/prof_$1 -name "*results.db" | head -1) > $O/kernel_stats_$1.csv
}
prof per_round "" || exit $?
prof on_g1 "--scheme bls-unchained-on-g1" || exit $?
prof recover "--mode recover" || exit $?
step traffic
TAG=$TAG/traffic bash tools/gpu/traffic.sh > $O/traffic.log 2>&1 || exit $?
echo done
