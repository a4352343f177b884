#!/bin/bash
# A/B: bench each library variant listed in $VARIANTS (paths relative to repo), same process settings.
export TMPDIR=/tmp
TAG=${TAG:-ab}
mkdir -p gpurun_out/$TAG
for v in $VARIANTS; do
  name=$(basename $v .so)
  DRAND_GPU_LIB=$PWD/$v timeout -k 10 600 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/$TAG/$name.json 2> gpurun_out/$TAG/$name.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/$TAG/$name.json')); print('$name', round(d['value']), d['verdict_mismatches'], {k: round(v,1) for k,v in d['roofline']['stage_ms'].items()})"
done
