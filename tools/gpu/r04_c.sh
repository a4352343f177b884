#!/bin/bash
# Round-4 session c: engine chunk size A/B on the headline workload (10M
# chained per round, --no-legs --no-rlc): 512Ki rounds per chunk (default)
# vs 640Ki (5M per lane = 8 chunks, no partial one) vs 1Mi, 2 reps.
export TMPDIR=/tmp
TAG=r04c1 REPS=2 VARIANTS="c512=X c640=DGPU_ENG_CHUNK=655360 c1m=DGPU_ENG_CHUNK=1048576" BENCH_ARGS="--steps 3 --no-cpu-baseline --no-e2e --no-legs --no-rlc" BENCH_T=400 bash tools/gpu/r04_ab.sh || exit $?
echo done
