#!/bin/bash
# Round-4 closing session: 1Mi engine chunks -- GPU suite + smoke, the default
# bench (every leg), and the rocprofv3 kernel-trace statistics of the headline
# command (the roofline kernel's per-launch check).
export TMPDIR=/tmp
O=gpurun_out/r04zzz
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
echo "== rocprof $(date +%T)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o bench -- python3 bench.py --no-cpu-baseline --no-e2e --no-legs --steps 2 > $O/prof.out 2>&1 || exit $?
python3 tools/rocpd_stats.py $(find $O/prof -name "*results.db" | head -1) > $O/kernel_stats.csv || true
echo done
