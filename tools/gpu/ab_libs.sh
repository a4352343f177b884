export TMPDIR=/tmp
O=gpurun_out/r02d; mkdir -p $O
for v in base pf sk pfsk; do
  if [ $v = base ]; then L=drand_amd/libdrand_gpu.so; else L=drand_amd/libdrand_gpu_$v.so; fi
  DRAND_GPU_LIB=$PWD/$L timeout -k 10 200 python -u bench.py --rounds 1000000 --steps 4 --no-cpu-baseline --no-e2e > $O/ab_$v.json 2> $O/ab_$v.err || exit $?
  echo $v done
done
