#!/bin/bash
# Round-4 session f: the full GPU suite on the localize + fused-Karabina +
# inlined-G1-decode build, then same-box A/Bs (each a separate bench.py run
# with its own time limit, stopping at the first failure):
#   f1 chained per-round 2M: fused Karabina (head) vs DGPU_KB_DEC=separate
#   f2 chained 10M RLC mode: localize-then-confirm (head) vs DGPU_RLC_LOCALIZE=0
#   f3 on-G1 10M per-round + RLC: inlined G1 decode vs libdrand_gpu_prev.so
#   f4 recovery 100k: head vs prev (k_recover_rlc_g1 at 2 waves/SIMD)
#   f5 microbenches: G2 decode with membership, RLC leaf window width
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
O=gpurun_out/r04f
mkdir -p $O
if [ -z "$NOTEST" ]; then
step pytest
timeout -k 10 720 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
fi
TAG=r04f1 VARIANTS="head=X sep=DGPU_KB_DEC=separate" bash tools/gpu/r04_ab.sh || exit $?
TAG=r04f2 VARIANTS="head=X noloc=DGPU_RLC_LOCALIZE=0" BENCH_ARGS="--mode rlc --steps 3 --no-cpu-baseline --no-e2e --no-legs" bash tools/gpu/r04_ab.sh || exit $?
TAG=r04f3 REPS=1 VARIANTS="head=X prev=LIB=libdrand_gpu_prev.so" BENCH_ARGS="--scheme bls-unchained-on-g1 --steps 2 --no-cpu-baseline --no-e2e --no-legs" bash tools/gpu/r04_ab.sh || exit $?
TAG=r04f4 REPS=1 VARIANTS="head=X prev=LIB=libdrand_gpu_prev.so" BENCH_ARGS="--mode recover --steps 3 --no-cpu-baseline" bash tools/gpu/r04_ab.sh || exit $?
step micro
timeout -k 10 200 tools/engbench/dec_g2_bin 2097152 > $O/dec_g2.txt 2>&1 || exit $?
timeout -k 10 200 tools/engbench/leaves_bin 2097152 > $O/leaves.txt 2>&1 || exit $?
cat $O/dec_g2.txt $O/leaves.txt
echo done
