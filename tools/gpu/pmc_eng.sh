#!/bin/bash
# PMC passes over the per-round verify pipeline (each its own rocprofv3 run, kernel-trace only).
export TMPDIR=/tmp
TAG=${TAG:-pmc_eng}
mkdir -p gpurun_out/$TAG
run() {  # name, counters
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $2 -d gpurun_out/$TAG/$1 -o p -- python3 tools/prof_verify.py --rounds 131072 --iters 1 > gpurun_out/$TAG/$1.log 2>&1
}
run sq1 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU" || exit $?
run sq2 "SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC" || exit $?
run sq3 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT" || exit $?
python3 tools/pmc_summary.py gpurun_out/$TAG
