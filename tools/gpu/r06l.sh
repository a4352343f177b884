# round 6 session l: the decoders' G2 membership test on the cofactor ladder's
# structure (lazy doublings, fast mixed additions of the stored point;
# default) vs g2_in_subgroup with the point in registers (-DDG_SUBGROUP_GENERIC):
# RLC pass (decode with membership up front) and threshold recovery (partials'
# decode); then the decode / RLC / recovery GPU tests
D=drand_amd/libdrand_gpu.so; G=drand_amd/libdrand_gpu_subgen.so
TAG=r06l/rlc VARIANTS="$G@REP=1 $D@REP=1 $G@REP=2 $D@REP=2" \
  BENCH_ARGS="--rounds 2000000 --no-e2e --no-legs --steps 3" bash tools/gpu/session.sh ab && \
TAG=r06l/rec VARIANTS="$G@REP=1 $D@REP=1 $G@REP=2 $D@REP=2" \
  BENCH_ARGS="--mode recover --steps 3" bash tools/gpu/session.sh ab && \
TAG=r06l/t PYTEST_SEL="tests/test_gpu_decode_fuzz.py tests/test_gpu_rlc_msm.py tests/test_gpu_rlc_ranks.py tests/test_recover.py tests/test_gpu_boundary.py tests/test_gpu_parity.py" bash tools/gpu/session.sh pytest
