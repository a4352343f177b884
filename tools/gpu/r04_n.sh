#!/bin/bash
# Round-4 session n: RLC bucket accumulation with the next point's gather
# issued before the current addition (libdrand_gpu_pf.so) vs head, 10M
# chained RLC at 0.1% corrupted and on-G1 RLC.
export TMPDIR=/tmp
TAG=r04n1 REPS=2 VARIANTS="head=X pf=LIB=libdrand_gpu_pf.so" BENCH_ARGS="--mode rlc --steps 3 --no-cpu-baseline --no-e2e --no-legs" bash tools/gpu/r04_ab.sh || exit $?
TAG=r04n2 REPS=1 VARIANTS="head=X pf=LIB=libdrand_gpu_pf.so" BENCH_ARGS="--mode rlc --scheme bls-unchained-on-g1 --steps 3 --no-cpu-baseline --no-e2e --no-legs" bash tools/gpu/r04_ab.sh || exit $?
echo done
