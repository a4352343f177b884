#!/bin/bash
# Round-4 first session: GPU tests + smoke on HEAD, the pending same-box A/B
# of the M_XIL removal (HEAD vs libdrand_gpu_prev.so = 501e09a^ engine
# tables), then the PMC passes of the shipped per-round pipeline.
export TMPDIR=/tmp
TAG=${TAG:-r04a}
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
if [ -z "$NOTEST" ]; then
step pytest
timeout -k 10 720 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
step smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
fi
R=${ROUNDS:-2000000}
for rep in 1 2; do
for v in ${VARIANTS:-head=X prev=LIB=libdrand_gpu_prev.so}; do
  name=${v%%=*}; envs=${v#*=}
  step "bench $name $rep"
  (
    IFS=','; for e in $envs; do
      case $e in LIB=*) export DRAND_GPU_LIB=$PWD/drand_amd/${e#LIB=};; X) ;; *) export "$e";; esac
    done
    timeout -k 10 300 python -u bench.py --rounds $R --steps 4 --no-cpu-baseline --no-e2e --no-legs --no-rlc > $O/ab_${name}_$rep.json 2> $O/ab_${name}_$rep.err
  ) || exit $?
done
done
if [ -z "$NOPMC" ]; then
P=$O/pmc
mkdir -p $P
run() {  # name, counters
  step "pmc $1"
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $2 -d $P/$1 -o p -- python3 tools/prof_verify.py --rounds 131072 --iters 1 > $P/$1.log 2>&1
}
run sq1 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU" || exit $?
run sq2 "SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC" || exit $?
run sq3 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH GRBM_GUI_ACTIVE GRBM_COUNT" || exit $?
run fetch "FETCH_SIZE" || exit $?
run write "WRITE_SIZE" || exit $?
python3 tools/pmc_summary.py $P > $P/pmc_summary.txt
python3 tools/traffic_summary.py $P 131072 $P/traffic.json > $P/traffic.log
fi
echo done
