#!/bin/bash
# Round-4: per-round batches cut into more slices alternating between the two
# lanes (DGPU_LANE_SLICES), so more of the hash runs beside the other lane's
# engine chunks: the two-lane test (slices 2 and 5), then same-box A/B at 10M
# chained per round: 2 (default) / 4 / 8 slices, 2 reps.
export TMPDIR=/tmp
TAG=r04sl1 REPS=2 PYTEST_K="two_lane" VARIANTS="s2=X s4=DGPU_LANE_SLICES=4 s8=DGPU_LANE_SLICES=8" BENCH_ARGS="--steps 3 --no-cpu-baseline --no-e2e --no-legs --no-rlc" BENCH_T=400 bash tools/gpu/r04_ab.sh || exit $?
echo done
