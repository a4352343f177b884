#!/bin/bash
# Round-4 session o: GPU suite with the lane-kernel threshold restricted to
# the RLC node checks (per-round calls keep the per-thread kernels at every
# size), then the chained 10M RLC bench at 0.1% corrupted.
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
O=gpurun_out/r04o
mkdir -p $O
step pytest
timeout -k 10 720 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
step rlc
timeout -k 10 300 python -u bench.py --mode rlc --steps 3 --no-cpu-baseline --no-e2e --no-legs > $O/rlc.json 2> $O/rlc.err || exit $?
head -c 200 $O/rlc.json; echo
echo done
