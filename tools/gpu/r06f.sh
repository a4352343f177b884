# round 6 session f: (1) the Karabina chain's twist of 2 f2 f5 from the product
# components (two reductions fewer per compressed squaring) vs reduced first;
# (2) k_lines_thr with a pair per wave (G1 point in SGPRs) vs both pairs per
# wave (A/B build, DGPU_LINES_WAVE); (3) the 8-context staging rehearsal
# (A/B build: stage-only hook); tests
A=drand_amd/libdrand_gpu_xired.so; B=drand_amd/libdrand_gpu_xinew.so; C=drand_amd/libdrand_gpu_ab.so
TAG=r06f VARIANTS="$A@REP=1 $B@REP=1 $A@REP=2 $B@REP=2 $C@DGPU_LINES_WAVE=0@REP=1 $C@DGPU_LINES_WAVE=1@REP=1 $C@DGPU_LINES_WAVE=0@REP=2 $C@DGPU_LINES_WAVE=1@REP=2" \
  BENCH_ARGS="--rounds 2000000 --no-e2e --no-rlc --no-legs --steps 3" bash tools/gpu/session.sh ab && \
TAG=r06f/kb PYTEST_SEL="tests/test_gpu_parity.py tests/test_gpu_ragged.py tests/test_gpu_g1.py tests/test_recover.py" bash tools/gpu/session.sh pytest && \
mkdir -p gpurun_out/r06f && DRAND_GPU_LIB=$PWD/drand_amd/libdrand_gpu_ab.so DGPU_MULTI_ALLOW_SAME_DEVICE=1 DGPU_TEST_STAGE_ONLY=1 \
  DGPU_ENG_CHUNK=131072 timeout -k 10 400 python -u tools/stage_rehearsal.py > gpurun_out/r06f/stage_rehearsal.json \
  2> gpurun_out/r06f/stage_rehearsal.err && head -c 800 gpurun_out/r06f/stage_rehearsal.json && echo && \
TAG=r06f/stg PYTEST_SEL="tests/test_gpu_boundary.py -k staged" bash tools/gpu/session.sh pytest
