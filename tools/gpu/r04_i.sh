#!/bin/bash
# Round-4 session i: GPU suite on the divstep-inversion + fused Karabina build,
# then same-box A/Bs at 2M chained per-round:
#   i1 head (k_kb_chain_dec_thr: chain + norms + per-thread divstep inversion
#      + decompression) vs sep (DGPU_KB_DEC=separate: chain, kb_norm, batched
#      inversion, kb_dec) vs conf (libdrand_gpu_conf.so: Fermat inversion)
#   i2 head vs l1 (libdrand_gpu_l1.so: k_lines_thr at 1 wave/SIMD, no spills)
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
O=gpurun_out/r04i
mkdir -p $O
if [ -z "$NOTEST" ]; then
step pytest
timeout -k 10 720 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
fi
TAG=r04i1 VARIANTS="head=X sep=DGPU_KB_DEC=separate conf=LIB=libdrand_gpu_conf.so" bash tools/gpu/r04_ab.sh || exit $?
TAG=r04i2 VARIANTS="head=X l1=LIB=libdrand_gpu_l1.so" bash tools/gpu/r04_ab.sh || exit $?
echo done
