#!/bin/bash
# Round-4 session z: small per-round batches on the lane kernels.  For n in
# 4Ki..256Ki rounds (per-round, --no-rlc), same box: head (per-thread lines /
# chain at every size), tg (libdrand_gpu_tg.so: chunks under 64Ki items on the
# 12-lane lines and 8-lane chain), tg with DGPU_THR_MIN=262144 and with
# DGPU_THR_MIN=1073741824 (lane kernels at every size).
export TMPDIR=/tmp
O=gpurun_out/r04z
mkdir -p $O
for n in 4096 16384 65536 131072 262144; do
  for v in head tg tg256 tgall; do
    echo "== n=$n $v $(date +%T)"
    (
      case $v in
        head) ;;
        tg) export DRAND_GPU_LIB=$PWD/drand_amd/libdrand_gpu_tg.so ;;
        tg256) export DRAND_GPU_LIB=$PWD/drand_amd/libdrand_gpu_tg.so DGPU_THR_MIN=262144 ;;
        tgall) export DRAND_GPU_LIB=$PWD/drand_amd/libdrand_gpu_tg.so DGPU_THR_MIN=1073741824 ;;
      esac
      timeout -k 10 200 python -u bench.py --rounds $n --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-legs --no-rlc > $O/b_${n}_$v.json 2> $O/b_${n}_$v.err
    ) || exit $?
  done
done
echo done
