#!/bin/bash
# Build engbench variants: build.sh NAME "-DFLAG ..." [NAME "-D..."]...
set -e
cd "$(dirname "$0")"
while [ $# -ge 2 ]; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 $2 -o "engbench_$1" engbench.hip
  shift 2
done
