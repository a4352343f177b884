#!/bin/bash
# A/B session: engine op microbench for every built tools/engbench variant,
# then the per-round bench on each library in $VARIANTS (alternating, two
# passes; stage ms per $ROUNDS rounds).  Optional GPU parity suite first
# (TEST=1).  Stops at the first failure.
export TMPDIR=/tmp
TAG=${TAG:-r02_ab2}
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
if [ -n "$TEST" ]; then
step pytest
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
fi
for b in tools/engbench/engbench_*; do
  [ -e "$b" ] || continue
  v=${b##*/engbench_}
  step "engbench $v"
  ENGBENCH_ONLY=${ENGBENCH_ONLY:-LDBL,LADD,M_SQR,M_LM1,E_CYC_chain,E_MUL} timeout -k 10 120 $b ${REPS:-64} > $O/engbench_$v.jsonl || exit $?
  cat $O/engbench_$v.jsonl
done
for pass in 1 2; do
  for v in $VARIANTS; do
    name=$(basename $v .so)
    step "bench $name pass $pass"
    DRAND_GPU_LIB=$PWD/$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e ${RLC:---no-rlc} --rounds ${ROUNDS:-2000000} --steps 3 > $O/${name}_$pass.json 2> $O/${name}_$pass.err || exit $?
    python3 -c "import json; d=json.load(open('$O/${name}_$pass.json')); print('$name', round(d['value']), d['verdict_mismatches'], {k: round(v,1) for k,v in d['stage_ms'].items()}, 'rlc', round(d['rlc']['value']) if d.get('rlc') else None)"
  done
done
echo done
