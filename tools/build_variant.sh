#!/bin/bash
# Build libdrand_gpu.so of another git revision (A/B baselines), in-tree:
#   bash tools/build_variant.sh <rev> <out.so> [extra hipcc flags]
# e.g. bash tools/build_variant.sh HEAD drand_amd/libdrand_gpu_prev.so
set -e
rev=$1; out=$2; shift 2
tmp=$(mktemp -d)
git archive "$rev" drand_amd/csrc include | tar -x -C "$tmp"
hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC "$@" -o "$out" "$tmp/drand_amd/csrc/capi.hip"
rm -rf "$tmp"
echo "built $out from $rev"
