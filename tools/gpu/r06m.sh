# round 6 session m: the recovery MSM's window additions on the ladder's
# structure (lazy doublings, fast mixed additions of the fetched entry, the
# generic slice only on an exceptional addition; default) vs the generic
# mixed addition throughout (-DDG_RECOVER_MSM_GENERIC); recovery tests on both
D=drand_amd/libdrand_gpu.so; G=drand_amd/libdrand_gpu_recgen.so
TAG=r06m VARIANTS="$G@REP=1 $D@REP=1 $G@REP=2 $D@REP=2 $G@REP=3 $D@REP=3" \
  BENCH_ARGS="--mode recover --steps 3" bash tools/gpu/session.sh ab && \
TAG=r06m/t PYTEST_SEL="tests/test_recover.py tests/test_gpu_defaults.py" bash tools/gpu/session.sh pytest && \
DRAND_GPU_LIB=$PWD/$G TAG=r06m/tg PYTEST_SEL="tests/test_recover.py" bash tools/gpu/session.sh pytest
