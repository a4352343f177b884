#!/bin/bash
# Same-box A/B: optional GPU tests (PYTEST_K subset), then bench.py with
# BENCH_ARGS for each variant in VARIANTS (name=ENV1,ENV2 or name=LIB=<file>
# or name=X for the default build), REPS repetitions, one JSON per run
# (ab_<name>_<rep>.json).  Each GPU step has its own time limit.
export TMPDIR=/tmp
TAG=${TAG:-r04ab}
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
if [ -n "$PYTEST_K" ]; then
step pytest
timeout -k 10 ${TEST_T:-600} python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread -k "$PYTEST_K" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
fi
for rep in $(seq 1 ${REPS:-2}); do
for v in ${VARIANTS:-head=X}; do
  name=${v%%=*}; envs=${v#*=}
  step "bench $name $rep"
  (
    for e in ${envs//,/ }; do
      case $e in LIB=*) export DRAND_GPU_LIB=$PWD/drand_amd/${e#LIB=};; X) ;; *) export "$e";; esac
    done
    timeout -k 10 ${BENCH_T:-300} python -u bench.py ${BENCH_ARGS:---rounds 2000000 --steps 4 --no-cpu-baseline --no-e2e --no-legs --no-rlc} > $O/ab_${name}_$rep.json 2> $O/ab_${name}_$rep.err
  ) || exit $?
done
done
echo done
