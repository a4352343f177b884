#!/bin/bash
# Round-4 session r: RLC bucket accumulation with the next point's index loaded
# one iteration ahead (libdrand_gpu_ia.so, DG_MSM_IDX_AHEAD) vs head: chained
# 10M RLC at 0.1% corrupted (2 reps) and on-G1 10M RLC.
export TMPDIR=/tmp
TAG=r04r1 REPS=2 VARIANTS="head=X ia=LIB=libdrand_gpu_ia.so" BENCH_ARGS="--mode rlc --steps 3 --no-cpu-baseline --no-e2e --no-legs" bash tools/gpu/r04_ab.sh || exit $?
TAG=r04r2 REPS=1 VARIANTS="head=X ia=LIB=libdrand_gpu_ia.so" BENCH_ARGS="--mode rlc --scheme bls-unchained-on-g1 --steps 3 --no-cpu-baseline --no-e2e --no-legs" bash tools/gpu/r04_ab.sh || exit $?
echo done
