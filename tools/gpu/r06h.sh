# round 6 session h: occupancy probe of the out-of-line Fp calls (1..8 waves
# per SIMD); kernel-trace profile and HBM traffic of the shipped library
mkdir -p gpurun_out/r06h && timeout -k 10 120 ./tools/engbench/powprobe_bin > gpurun_out/r06h/powprobe.json && \
  cat gpurun_out/r06h/powprobe.json && \
TAG=r06h bash tools/gpu/session.sh prof traffic
