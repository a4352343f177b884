# round 6 session s: the T-step doubling's X and Z leaving with their first
# coefficient unreduced (two reductions fewer; default) vs both reduced
# (-DDG_LINES_DBL_PLAIN); the lines / membership / parity GPU tests
D=drand_amd/libdrand_gpu.so; P=drand_amd/libdrand_gpu_linesplain.so
TAG=r06s VARIANTS="$P@REP=1 $D@REP=1 $P@REP=2 $D@REP=2 $P@REP=3 $D@REP=3" \
  BENCH_ARGS="--rounds 2000000 --no-e2e --no-rlc --no-legs --steps 3" bash tools/gpu/session.sh ab && \
TAG=r06s/t PYTEST_SEL="tests/test_gpu_parity.py tests/test_gpu_ragged.py tests/test_gpu_large.py tests/test_gpu_decode_fuzz.py" bash tools/gpu/session.sh pytest
