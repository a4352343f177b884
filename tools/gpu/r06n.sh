# round 6 session n: the RLC root MSM's G2 bucket sums with fast mixed
# additions of the fetched row (generic redo of a thread's range on an
# exceptional addition; default) vs the generic mixed addition (-DDG_MSM_GENERIC)
D=drand_amd/libdrand_gpu.so; G=drand_amd/libdrand_gpu_msmgen.so
TAG=r06n VARIANTS="$G@REP=1 $D@REP=1 $G@REP=2 $D@REP=2" \
  BENCH_ARGS="--rounds 10000000 --no-e2e --no-legs --steps 3" bash tools/gpu/session.sh ab && \
TAG=r06n/t PYTEST_SEL="tests/test_gpu_rlc_msm.py tests/test_gpu_rlc_ranks.py tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_large.py" bash tools/gpu/session.sh pytest
