# round 6 last check of the final tree: whole GPU suite, smoke, default bench
TAG=r06z bash tools/gpu/session.sh pytest smoke bench
