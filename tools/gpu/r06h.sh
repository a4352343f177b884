# round 6 session h: occupancy probe of the out-of-line Fp calls (1..8 waves
# per SIMD); kernel-trace profile and HBM traffic of the shipped library
mkdir -p gpurun_out/r06h && hipcc --offload-arch=gfx950 -O3 -std=c++17 -o /tmp/powprobe_bin tools/engbench/powprobe.hip && timeout -k 10 120 /tmp/powprobe_bin > gpurun_out/r06h/powprobe.json && \
  cat gpurun_out/r06h/powprobe.json && \
TAG=r06h bash tools/gpu/session.sh prof traffic
