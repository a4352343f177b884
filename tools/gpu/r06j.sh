# round 6 session j: the Karabina chain on two lanes per round
# (k_kb_chain_pair, 168 VGPRs, 3 waves/SIMD; A/B build DGPU_KB_PAIR=1) vs one
# thread per round (256 VGPRs, 2 waves), and the pair kernel forced to 4 waves
# (-DDG_KB_PAIR_OCC=4); parity of the pair kernel
A=drand_amd/libdrand_gpu_ab.so; A4=drand_amd/libdrand_gpu_ab_pair4.so
TAG=r06j VARIANTS="$A@DGPU_KB_PAIR=0@REP=1 $A@DGPU_KB_PAIR=1@REP=1 $A4@DGPU_KB_PAIR=1@REP=1 $A@DGPU_KB_PAIR=0@REP=2 $A@DGPU_KB_PAIR=1@REP=2 $A4@DGPU_KB_PAIR=1@REP=2" \
  BENCH_ARGS="--rounds 2000000 --no-e2e --no-rlc --no-legs --steps 3" bash tools/gpu/session.sh ab && \
TAG=r06j/kb PYTEST_SEL="tests/test_gpu_parity.py -k karabina" bash tools/gpu/session.sh pytest
