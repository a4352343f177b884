#!/bin/bash
# Run every built engbench variant (GPU box).  Output: gpurun_out/$TAG/<variant>.jsonl
TAG=${TAG:-engbench}
mkdir -p gpurun_out/$TAG
for b in tools/engbench/engbench_*; do
  v=${b##*/engbench_}
  timeout -k 10 120 $b ${REPS:-64} > gpurun_out/$TAG/$v.jsonl || exit $?
  echo "== $v"; cat gpurun_out/$TAG/$v.jsonl
done
