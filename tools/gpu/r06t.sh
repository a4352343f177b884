# round 6 session t: g2_clear_cofactor (RLC node checks, hash_to_g2, the
# finish's exceptional redo) as a register ladder with lazy doublings and fast
# additions, the generic form on an exceptional case (default) vs the generic
# form always (-DDG_COFACTOR_GENERIC): the RLC pass at 10M (k_rlc_prep); the
# whole GPU suite and smoke on the default
D=drand_amd/libdrand_gpu.so; G=drand_amd/libdrand_gpu_cofgen.so
TAG=r06t VARIANTS="$G@REP=1 $D@REP=1 $G@REP=2 $D@REP=2" \
  BENCH_ARGS="--rounds 10000000 --no-e2e --no-legs --steps 3" bash tools/gpu/session.sh ab && \
TAG=r06t/all bash tools/gpu/session.sh pytest smoke
