#!/bin/bash
# Round-4 session j: GPU suite on the split Karabina decompression (norms and
# decompression parts at the chain's snaps, k_kb_chain_pre_thr; one thread per
# round inverting by divsteps and decompressing, k_kb_dec_thr), then same-box
# A/B at 2M chained per-round: head vs sep (DGPU_KB_DEC=separate: kb_norm,
# batched divstep inversion, kb_dec) vs d1 (libdrand_gpu_d1.so: k_kb_dec_thr
# at 1 wave/SIMD).
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
O=gpurun_out/r04j
mkdir -p $O
if [ -z "$NOTEST" ]; then
step pytest
timeout -k 10 720 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
fi
TAG=r04j1 VARIANTS="head=X sep=DGPU_KB_DEC=separate d1=LIB=libdrand_gpu_d1.so" bash tools/gpu/r04_ab.sh || exit $?
echo done
