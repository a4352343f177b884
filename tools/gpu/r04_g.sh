#!/bin/bash
# Round-4 session g: GPU suite + smoke on the shipped build, the RLC descent
# step A/B (levels per descent step: 5 = round 3's, 3, 2) on the 10M chained
# chain at 0.1% corrupted, then the default bench (every BASELINE config leg).
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
O=gpurun_out/r04g
mkdir -p $O
if [ -z "$NOTEST" ]; then
step pytest
timeout -k 10 720 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
step smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
fi
if [ -z "$NOAB" ]; then
TAG=r04g1 REPS=1 VARIANTS="d5=DGPU_RLC_DESCENT_STEP=5 d3=DGPU_RLC_DESCENT_STEP=3 d2=DGPU_RLC_DESCENT_STEP=2" BENCH_ARGS="--mode rlc --steps 3 --no-cpu-baseline --no-e2e --no-legs" bash tools/gpu/r04_ab.sh || exit $?
fi
if [ -z "$NOBENCH" ]; then
step bench
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
head -c 300 $O/bench.json; echo
fi
echo done
