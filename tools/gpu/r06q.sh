# round 6 session q: G1 additions (Jacobian and mixed) with lazy linear steps
# (g1addnew) vs every step reduced (-DDG_G1_ADD_PLAIN): on-G1 per round and
# RLC (G1 bucket sums, tree, cofactor and membership ladders); G1 tests
N=drand_amd/libdrand_gpu_g1addnew.so; P=drand_amd/libdrand_gpu_g1addplain.so
TAG=r06q VARIANTS="$P@REP=1 $N@REP=1 $P@REP=2 $N@REP=2" \
  BENCH_ARGS="--scheme bls-unchained-on-g1 --rounds 10000000 --no-e2e --no-legs --steps 3" bash tools/gpu/session.sh ab && \
DRAND_GPU_LIB=$PWD/$N TAG=r06q/t PYTEST_SEL="tests/test_gpu_g1.py tests/test_gpu_decode_fuzz.py tests/test_gpu_rlc_msm.py tests/test_gpu_rlc_ranks.py tests/test_gpu_multi.py" bash tools/gpu/session.sh pytest
