# round 6: the default bench on the exact final tree
TAG=r06zz bash tools/gpu/session.sh bench
