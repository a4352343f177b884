# round 6 session p: the 11-isogeny's four polynomials in one lazy Horner pass
# (D^s shared, sums unreduced; iso11new) vs four passes, every sum reduced
# (-DDG_ISO11_PLAIN); both with the lazy G1 doubling: bls-unchained-on-g1 per
# round and RLC
N=drand_amd/libdrand_gpu_iso11new.so; P=drand_amd/libdrand_gpu_iso11plain.so
TAG=r06p VARIANTS="$P@REP=1 $N@REP=1 $P@REP=2 $N@REP=2" \
  BENCH_ARGS="--scheme bls-unchained-on-g1 --rounds 2000000 --no-e2e --no-legs --steps 3" bash tools/gpu/session.sh ab && \
DRAND_GPU_LIB=$PWD/$N TAG=r06p/t PYTEST_SEL="tests/test_gpu_g1.py tests/test_gpu_decode_fuzz.py" bash tools/gpu/session.sh pytest
