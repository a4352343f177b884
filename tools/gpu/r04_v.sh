#!/bin/bash
# Round-4 session v: the Karabina planes with the compressed components first
# (kb_pos: f1, f2, f4, f5 in one 32-byte run per round and limb, f0, f3 in one
# 16-byte run; dwordx4 loads/stores in the chain and the decompression): the
# Karabina / ragged / parity GPU tests, then same-box A/B vs
# libdrand_gpu_prev.so (component order) at 2M chained per-round, 2 reps.
export TMPDIR=/tmp
TAG=r04v1 REPS=2 PYTEST_K="karabina or ragged or parity or g1 or recover" VARIANTS="head=X prev=LIB=libdrand_gpu_prev.so" bash tools/gpu/r04_ab.sh || exit $?
echo done
