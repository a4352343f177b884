# round 6 session e: staging (message parts first, per-slice record checks) --
# boundary / parity / multi tests, the default bench without legs (end-to-end
# vs resident), the 8-context staging rehearsal
TAG=r06e PYTEST_SEL="tests/test_gpu_boundary.py tests/test_gpu_multi.py tests/test_gpu_parity.py" \
  bash tools/gpu/session.sh pytest && \
TAG=r06e BENCH_ARGS="--no-legs --no-rlc" bash tools/gpu/session.sh bench && \
TAG=r06e bash tools/gpu/session.sh abi8
