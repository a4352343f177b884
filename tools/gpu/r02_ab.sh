#!/bin/bash
# Round-2 engine A/B session: GPU parity suite on the shipped library, the
# engine op microbench, then the per-round bench on each library variant in
# $VARIANTS (alternating, two passes).  Stops at the first failure.
export TMPDIR=/tmp
TAG=${TAG:-r02_ab}
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
if [ -z "$NO_TEST" ]; then
step pytest
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
fi
step engbench
ENGBENCH_ONLY=${ENGBENCH_ONLY:-E_CYC,E_CYC_fast,E_MUL,M_SQR,LDBL} timeout -k 10 120 tools/engbench/engbench_base > $O/engbench.jsonl || exit $?
cat $O/engbench.jsonl
for pass in 1 2; do
  for v in $VARIANTS; do
    name=$(basename $v .so)
    step "bench $name pass $pass"
    DRAND_GPU_LIB=$PWD/$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e --no-rlc --rounds ${ROUNDS:-2000000} --steps 3 > $O/${name}_$pass.json 2> $O/${name}_$pass.err || exit $?
    python3 -c "import json; d=json.load(open('$O/${name}_$pass.json')); print('$name', round(d['value']), d['verdict_mismatches'], {k: round(v,1) for k,v in d['stage_ms'].items()})"
  done
done
echo done
