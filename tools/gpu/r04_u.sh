#!/bin/bash
# Round-4 session u: Fp reductions inlined in the per-thread kernels' step
# formulas (no out-of-line call): ci = the Karabina chain's 10 reductions per
# compressed squaring (libdrand_gpu_ci.so), li = the T-step doubling's 6
# (libdrand_gpu_li.so), vs head; chained per-round 2M rounds, 2 reps.
export TMPDIR=/tmp
TAG=r04u1 REPS=2 VARIANTS="head=X ci=LIB=libdrand_gpu_ci.so li=LIB=libdrand_gpu_li.so" bash tools/gpu/r04_ab.sh || exit $?
echo done
