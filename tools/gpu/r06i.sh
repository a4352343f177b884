# round 6 session i: (1) the SSWU stage in five launches with both
# exponentiations on a 90-VGPR kernel (default) vs the fused 256-VGPR kernel
# (-DDG_SSWU_FUSED); (2) occupancy screen of the per-thread kernels (chain,
# lines, Karabina decompression, cofactor ladder) at 3 and 4 waves per SIMD;
# then the whole GPU suite on the default library
D=drand_amd/libdrand_gpu.so; F=drand_amd/libdrand_gpu_sswufused.so; O3=drand_amd/libdrand_gpu_occ3.so; O4=drand_amd/libdrand_gpu_occ4.so
TAG=r06i VARIANTS="$F@REP=1 $D@REP=1 $O3@REP=1 $O4@REP=1 $F@REP=2 $D@REP=2 $O3@REP=2 $O4@REP=2" \
  BENCH_ARGS="--rounds 2000000 --no-e2e --no-legs --steps 3" bash tools/gpu/session.sh ab && \
TAG=r06i/all bash tools/gpu/session.sh pytest
