# round 6 session o: the G1 doubling with lazy linear steps (7 products and 3
# reductions instead of 14; default) vs every step reduced (-DDG_G1_DBL_PLAIN):
# bls-unchained-on-g1 per round and RLC (hash to G1 and the G1 decoders'
# membership test run [|x|] ladders of G1 doublings); G1 tests
D=drand_amd/libdrand_gpu.so; P=drand_amd/libdrand_gpu_g1plain.so
TAG=r06o VARIANTS="$P@REP=1 $D@REP=1 $P@REP=2 $D@REP=2" \
  BENCH_ARGS="--scheme bls-unchained-on-g1 --rounds 2000000 --no-e2e --no-legs --steps 3" bash tools/gpu/session.sh ab && \
TAG=r06o/t PYTEST_SEL="tests/test_gpu_g1.py tests/test_gpu_decode_fuzz.py tests/test_gpu_boundary.py tests/test_recover.py tests/test_gpu_defaults.py" bash tools/gpu/session.sh pytest
