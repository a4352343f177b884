#!/bin/bash
# One GPU session: parity suite, the 10M bench (+ DGPU_SUBGROUP=decode A/B on
# 1M rounds), rocprofv3 kernel stats of the bench, then the PMC passes.
# Stops at the first failure.
export TMPDIR=/tmp
TAG=${TAG:-r02b}
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step pytest
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
step bench
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
head -c 1500 $O/bench.json; echo
if [ -z "$NO_AB" ]; then
step bench-ab-1M
timeout -k 10 300 python -u bench.py --rounds 1000000 --steps 3 --no-cpu-baseline --no-e2e > $O/bench_1M.json 2> $O/bench_1M.err || exit $?
DGPU_SUBGROUP=decode timeout -k 10 300 python -u bench.py --rounds 1000000 --steps 3 --no-cpu-baseline --no-e2e > $O/bench_1M_decodesub.json 2> $O/bench_1M_decodesub.err || exit $?
fi
[ -n "$NO_PROF" ] && exit 0
step rocprof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o bench -- python3 bench.py --no-cpu-baseline --no-e2e --steps 2 > $O/prof.out 2>&1 || exit $?
python3 tools/rocpd_stats.py $(find $O/prof -name "*results.db" | head -1) > $O/kernel_stats.csv
[ -n "$NO_PMC" ] && exit 0
TAG=$TAG/pmc bash tools/gpu/r02_pmc_only.sh || exit $?
echo done
