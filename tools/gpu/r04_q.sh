#!/bin/bash
# Round-4 session q, the build to ship (MSM run 8, RLC-only lane threshold): GPU suite + smoke, the default bench
# (every BASELINE config leg), rocprofv3 kernel-trace statistics of the
# headline command and the PMC passes (one rocprofv3 run per pass, kernel
# trace only).
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
O=gpurun_out/r04q
mkdir -p $O
step pytest
timeout -k 10 720 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
step smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
step bench
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
head -c 300 $O/bench.json; echo
HTAG=r04q NOAB=1 bash tools/gpu/r04_h.sh 2>&1 | sed 's/^/[h] /'
