#!/bin/bash
# PMC passes (each its own rocprofv3 run, kernel-trace only; no sys/runtime
# trace; at most 8 SQ counters a pass).  HBM bytes: tools/gpu/session.sh traffic.
export TMPDIR=/tmp
TAG=${TAG:-pmc}
mkdir -p gpurun_out/$TAG
run() {  # name, counters
  timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv --pmc $2 -d gpurun_out/$TAG/$1 -o p -- python3 tools/prof_verify.py ${PROF_ARGS} > gpurun_out/$TAG/$1.log 2>&1
}
run sq1 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU" || exit $?
run sq2 "SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH" || exit $?
# VALU instruction classes (v_mad_u64_u32 counts as INT64) and LDS conflicts
run sq3 "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" || exit $?
run tcc "TCC_HIT_sum TCC_MISS_sum" || exit $?
python3 tools/pmc_summary.py gpurun_out/$TAG > gpurun_out/$TAG/pmc_summary.txt
echo done
