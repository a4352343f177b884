#!/bin/bash
# RLC mode A/B (configs[2]): GPU tests, then bench --mode rlc at 10M rounds
# (0.1% and 0% corrupted) for each library variant (name=LIB=<file> or X).
export TMPDIR=/tmp
TAG=${TAG:-r03q}
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
if [ -z "$NOTEST" ]; then
step pytest
timeout -k 10 600 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
fi
for rep in 1 2; do
for v in ${VARIANTS:-new=X}; do
  name=${v%%=*}; e=${v#*=}
  for cr in 0.001 0; do
    step "rlc $name $cr"
    (
      case $e in LIB=*) export DRAND_GPU_LIB=$PWD/drand_amd/${e#LIB=};; esac
      timeout -k 10 300 python -u bench.py --mode rlc --rounds 10000000 --corrupt-rate $cr --steps 3 --no-cpu-baseline --no-e2e --no-legs > $O/rlc_${name}_${cr}_$rep.json 2> $O/rlc_${name}_${cr}_$rep.err
    ) || exit $?
  done
done
done
echo done
