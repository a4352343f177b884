#!/bin/bash
# Hash/decode rework check: GPU parity suite, 1M and 10M per-round benches
# (stage times), then the FETCH/WRITE passes for the traffic table.
export TMPDIR=/tmp
TAG=${TAG:-r02g}
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step pytest
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
step bench1M
timeout -k 10 300 python -u bench.py --rounds 1000000 --no-rlc --no-e2e > $O/bench_1M.json 2> $O/bench_1M.err || exit $?
step bench10M
timeout -k 10 600 python -u bench.py --no-rlc --no-e2e > $O/bench_10M.json 2> $O/bench_10M.err || exit $?
run() {  # name, counters
  step "pmc $1"
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $2 -d $O/$1 -o p -- python3 tools/prof_verify.py --rounds 131072 --iters 1 > $O/$1.log 2>&1
}
run fetch "FETCH_SIZE" || exit $?
run write "WRITE_SIZE" || exit $?
python3 tools/traffic_summary.py $O 131072 $O/traffic.json > $O/traffic.log
echo done
