# round 6 session r: the fast group-law paths' generic redo forced on every
# item (A/B build hook DGPU_TEST_FORCE_EXC=1), per round, RLC and recovery,
# then the whole GPU suite on the final libraries
TAG=r06r/redo PYTEST_SEL="tests/test_gpu_parity.py -k generic_redo tests/test_recover.py -k generic_redo" bash tools/gpu/session.sh pytest && \
TAG=r06r/all bash tools/gpu/session.sh pytest smoke
