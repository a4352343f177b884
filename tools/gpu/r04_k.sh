#!/bin/bash
# Round-4 session k: the Karabina test (default three-kernel decompression
# with the divstep inversion, and DGPU_KB_DEC=split), then same-box A/B of
# DGPU_THR_MIN (pairing chunks below it take the 12-lane lines and the 8-lane
# chain, which fill the chip at small sizes) on the 10M chained RLC leg at
# 0.1% corrupted (the localization's node checks are 10k-80k-item batches).
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
O=gpurun_out/r04k
mkdir -p $O
step pytest
timeout -k 10 400 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread -k "karabina or ragged or rlc" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
TAG=r04k1 REPS=2 VARIANTS="head=X t64=DGPU_THR_MIN=65536 t256=DGPU_THR_MIN=262144" BENCH_ARGS="--mode rlc --steps 3 --no-cpu-baseline --no-e2e --no-legs" bash tools/gpu/r04_ab.sh || exit $?
echo done
