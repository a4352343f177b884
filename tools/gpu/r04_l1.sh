#!/bin/bash
# Round-4: two lanes (streams over the batch halves, default) vs one lane
# (DGPU_LANES=1) with 1Mi-round engine chunks, 10M chained per round, 2 reps.
export TMPDIR=/tmp
TAG=r04l1 REPS=2 VARIANTS="two=X one=DGPU_LANES=1" BENCH_ARGS="--steps 3 --no-cpu-baseline --no-e2e --no-legs --no-rlc" BENCH_T=400 bash tools/gpu/r04_ab.sh || exit $?
echo done
