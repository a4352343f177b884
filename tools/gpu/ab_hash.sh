#!/bin/bash
# A/B of library builds on the per-round path (2M rounds), two rounds of
# alternation to expose run-to-run spread.
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r02h}; mkdir -p $O
for pass in 1 2; do
for v in ${VARIANTS:-old new dec4}; do
  if [ $v = new ]; then L=drand_amd/libdrand_gpu.so; else L=drand_amd/libdrand_gpu_$v.so; fi
  DRAND_GPU_LIB=$PWD/$L timeout -k 10 200 python -u bench.py --rounds 2000000 --steps 3 --no-cpu-baseline --no-e2e --no-rlc > $O/ab_${v}_$pass.json 2> $O/ab_${v}_$pass.err || exit $?
  echo $v $pass done
done
done
