#!/bin/bash
# Round-4 session s: the RLC tree-level kernel (k_rlc_level) bounded at 2
# waves/SIMD (libdrand_gpu_lv2.so) vs head (1 wave/SIMD, no spills): chained
# 10M RLC at 0.1% corrupted (2 reps).
export TMPDIR=/tmp
TAG=r04s1 REPS=2 VARIANTS="head=X lv2=LIB=libdrand_gpu_lv2.so" BENCH_ARGS="--mode rlc --steps 3 --no-cpu-baseline --no-e2e --no-legs" bash tools/gpu/r04_ab.sh || exit $?
echo done
