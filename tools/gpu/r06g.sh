# round 6 session g: (1) k_h2c_finish with its cold points parked in HBM and
# call-free ladders (default) vs the round-5 inline ladder (-DDG_FINISH_INL);
# (2) the lazy Karabina decompression (default) vs every step reduced
# (-DDG_KB_DEC_PLAIN); then the whole GPU suite
D=drand_amd/libdrand_gpu.so; F=drand_amd/libdrand_gpu_finl.so; K=drand_amd/libdrand_gpu_kbplain.so
TAG=r06g VARIANTS="$F@REP=1 $D@REP=1 $K@REP=1 $F@REP=2 $D@REP=2 $K@REP=2" \
  BENCH_ARGS="--rounds 2000000 --no-e2e --no-rlc --no-legs --steps 3" bash tools/gpu/session.sh ab && \
TAG=r06g/all bash tools/gpu/session.sh pytest
