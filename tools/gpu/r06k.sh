# round 6 session k: the cofactor ladder's doubling with four reductions
# fewer (Y3's product and Z carried unreduced; default) vs every doubling
# fully reduced (-DDG_LADDER_DBL_PLAIN); the hash-related GPU tests
D=drand_amd/libdrand_gpu.so; P=drand_amd/libdrand_gpu_dblplain.so
TAG=r06k VARIANTS="$P@REP=1 $D@REP=1 $P@REP=2 $D@REP=2 $P@REP=3 $D@REP=3" \
  BENCH_ARGS="--rounds 2000000 --no-e2e --no-rlc --no-legs --steps 3" bash tools/gpu/session.sh ab && \
TAG=r06k/h PYTEST_SEL="tests/test_gpu_parity.py tests/test_gpu_ragged.py tests/test_gpu_large.py" bash tools/gpu/session.sh pytest
