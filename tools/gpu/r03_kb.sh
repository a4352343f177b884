#!/bin/bash
# Karabina FE: GPU tests, then a same-box A/B of FE variants on the per-round
# headline pipeline, then rocprof kernel stats of the default build.  Each GPU
# step has its own time limit.  VARIANTS: space-separated name=ENV1,ENV2...
# (DGPU_FE=gs is the Granger-Scott kernel; LIB=<file> selects an in-tree build).
export TMPDIR=/tmp
TAG=${TAG:-r03h}
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
if [ -z "$NOTEST" ]; then
step pytest
timeout -k 10 600 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
fi
R=${ROUNDS:-2000000}
for rep in 1 2; do
for v in ${VARIANTS:-kb=X gs=DGPU_FE=gs}; do
  name=${v%%=*}; envs=${v#*=}
  step "bench $name"
  (
    IFS=','; for e in $envs; do
      case $e in LIB=*) export DRAND_GPU_LIB=$PWD/drand_amd/${e#LIB=};; X) ;; *) export "$e";; esac
    done
    timeout -k 10 300 python -u bench.py --rounds $R --steps 4 --no-cpu-baseline --no-e2e --no-legs --no-rlc > $O/ab_${name}_$rep.json 2> $O/ab_${name}_$rep.err
  ) || exit $?
done
done
if [ -n "$PROF" ]; then
step rocprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o bench -- python3 bench.py --rounds 1000000 --no-cpu-baseline --no-e2e --no-legs --no-rlc --steps 2 > $O/prof.out 2>&1 || exit $?
python3 tools/rocpd_stats.py $(find $O/prof -name "*results.db" | head -1) > $O/kernel_stats.csv
fi
echo done
