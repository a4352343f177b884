#!/bin/bash
# Round-4 GPU session: GPU tests (optionally a -k subset) + smoke, then the
# bench runs listed in BENCHES (";"-separated argument lists, one bench.py run
# each, written to bench_<i>.json), optionally a rocprofv3 kernel-stats pass.
# Each GPU step has its own time limit; the script stops at the first failure.
export TMPDIR=/tmp
TAG=${TAG:-r04b}
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
if [ -z "$NOTEST" ]; then
step pytest
timeout -k 10 ${TEST_T:-720} python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
step smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
fi
i=0
IFS=';' read -ra RUNS <<< "${BENCHES}"
for args in "${RUNS[@]}"; do
  [ -z "$args" ] && continue
  step "bench $i: $args"
  timeout -k 10 ${BENCH_T:-600} python -u bench.py $args > $O/bench_$i.json 2> $O/bench_$i.err || exit $?
  head -c 300 $O/bench_$i.json; echo
  i=$((i+1))
done
if [ -n "$PROF" ]; then
step rocprof
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o bench -- python3 bench.py $PROF > $O/prof.out 2>&1 || exit $?
python3 tools/rocpd_stats.py $(find $O/prof -name "*results.db" | head -1) > $O/kernel_stats.csv
fi
echo done
