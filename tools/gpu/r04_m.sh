#!/bin/bash
# Round-4 session m: RLC descent step A/B on the shipped build (small node
# checks now on the lane kernels): 10M chained at 0.1% corrupted, steps 3
# (default) / 2 / 1.
export TMPDIR=/tmp
TAG=r04m1 REPS=2 VARIANTS="d3=X d2=DGPU_RLC_DESCENT_STEP=2 d1=DGPU_RLC_DESCENT_STEP=1" BENCH_ARGS="--mode rlc --steps 3 --no-cpu-baseline --no-e2e --no-legs" bash tools/gpu/r04_ab.sh || exit $?
echo done
