#!/bin/bash
# Round-4 final session: GPU suite + smoke, then the default bench (every
# BASELINE config leg) on the shipped tree.
export TMPDIR=/tmp
O=gpurun_out/r04zz
mkdir -p $O
echo "== pytest $(date +%T)"
timeout -k 10 720 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
echo "== smoke $(date +%T)"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
echo "== bench $(date +%T)"
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
head -c 300 $O/bench.json; echo
echo done
