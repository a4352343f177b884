# round 6 closing run on the final tree: whole GPU suite, smoke, the default
# bench (every leg), kernel-trace profile and HBM traffic
TAG=${TAG:-r06final} bash tools/gpu/session.sh pytest smoke bench prof traffic
