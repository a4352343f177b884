#!/bin/bash
# Counter session: the PMC passes of the
# per-round pipeline (VALU / LDS / occupancy counters, HBM traffic), one
# rocprofv3 run per pass, kernel-trace only.  Stops at the first failure.
export TMPDIR=/tmp
TAG=${TAG:-r03_pmc}
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
run() {  # name, counters
  step "pmc $1"
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $2 -d $O/$1 -o p -- python3 tools/prof_verify.py --rounds 131072 --iters 1 > $O/$1.log 2>&1
}
run sq1 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU" || exit $?
run sq2 "SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC" || exit $?
run sq3 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH GRBM_GUI_ACTIVE GRBM_COUNT" || exit $?
run fetch "FETCH_SIZE" || exit $?
run write "WRITE_SIZE" || exit $?
python3 tools/pmc_summary.py $O > $O/pmc_summary.txt
python3 tools/traffic_summary.py $O 131072 $O/traffic.json > $O/traffic.log
echo done
