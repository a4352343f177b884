# round 6 session d: GPU suite + smoke, the engine-without-idle-lanes A/B
# (A/B build: DGPU_ENG_XW 0 / 1 Miller / 3 Miller + FE segments), then the default bench
A=drand_amd/libdrand_gpu_ab.so
TAG=r06d bash tools/gpu/session.sh pytest smoke && \
TAG=r06d VARIANTS="$A@DGPU_ENG_XW=0@REP=1 $A@DGPU_ENG_XW=1@REP=1 $A@DGPU_ENG_XW=3@REP=1 $A@DGPU_ENG_XW=0@REP=2 $A@DGPU_ENG_XW=1@REP=2 $A@DGPU_ENG_XW=3@REP=2" \
  BENCH_ARGS="--rounds 2000000 --no-e2e --no-rlc --no-legs --steps 3" bash tools/gpu/session.sh ab && \
TAG=r06d BENCH_ARGS="--no-legs" bash tools/gpu/session.sh bench
