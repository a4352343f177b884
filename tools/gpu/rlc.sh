#!/bin/bash
export TMPDIR=/tmp
TAG=${TAG:-rlc}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/$TAG/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/$TAG/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for m in per-round rlc; do
  timeout -k 10 600 python bench.py --no-cpu-baseline --mode $m ${BENCH_ARGS} > gpurun_out/$TAG/bench_$m.json 2> gpurun_out/$TAG/bench_$m.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/$TAG/bench_$m.json')); print('$m', round(d['value']), 'mism', d['verdict_mismatches'], {k: round(v,1) for k,v in d['stage_ms'].items()})"
done
