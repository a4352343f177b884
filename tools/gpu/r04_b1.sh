#!/bin/bash
# Round-4: RLC bucket accumulation (k_msm_bucket) at 1 wave/SIMD (no spills;
# libdrand_gpu_b1.so) vs 2 (head), chained 10M RLC at 0.1% and on-G1 10M RLC.
export TMPDIR=/tmp
TAG=r04b1 REPS=2 VARIANTS="head=X b1=LIB=libdrand_gpu_b1.so" BENCH_ARGS="--mode rlc --steps 3 --no-cpu-baseline --no-e2e --no-legs" bash tools/gpu/r04_ab.sh || exit $?
echo done
