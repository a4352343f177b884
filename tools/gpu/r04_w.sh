#!/bin/bash
# Round-4 session w: batched recovery MSM with radix-32 windows and [1..16]
# tables (libdrand_gpu_w5.so, DG_REC_W=5) vs radix-16 / [1..8] (head): the
# recovery GPU tests on the w5 build, then same-box A/B of --mode recover
# (100k rounds, 17 of 32), 2 reps.
export TMPDIR=/tmp
O=gpurun_out/r04w
mkdir -p $O
echo "== pytest w5 $(date +%T)"
DRAND_GPU_LIB=$PWD/drand_amd/libdrand_gpu_w5.so timeout -k 10 400 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread -k "recover" > $O/pytest_w5.log 2>&1
rc=$?; tail -3 $O/pytest_w5.log
[ $rc -ne 0 ] && exit $rc
TAG=r04w1 REPS=2 VARIANTS="head=X w5=LIB=libdrand_gpu_w5.so" BENCH_ARGS="--mode recover --steps 3 --no-cpu-baseline" bash tools/gpu/r04_ab.sh || exit $?
echo done
