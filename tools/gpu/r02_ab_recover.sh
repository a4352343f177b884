#!/bin/bash
# A/B session for the recovery path (configs[4]): optional GPU parity suite
# (TEST=1), then bench.py --mode recover on each library in $VARIANTS
# (alternating, two passes).  Stops at the first failure.
export TMPDIR=/tmp
TAG=${TAG:-r02_abr}
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
if [ -n "$TEST" ]; then
step pytest
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
fi
for pass in 1 2; do
  for v in $VARIANTS; do
    name=$(basename $v .so)
    step "recover $name pass $pass"
    DRAND_GPU_LIB=$PWD/$v timeout -k 10 300 python -u bench.py --mode recover --no-cpu-baseline --steps 3 > $O/${name}_$pass.json 2> $O/${name}_$pass.err || exit $?
    python3 -c "import json; d=json.load(open('$O/${name}_$pass.json')); print('$name', round(d['value']), d.get('verdict_mismatches'), {k: round(v,1) for k,v in d['stage_ms'].items()})"
  done
done
echo done
