#!/bin/bash
# PMC passes (each its own rocprofv3 run, kernel-trace only; no sys/runtime trace).
export TMPDIR=/tmp
TAG=${TAG:-pmc}
mkdir -p gpurun_out/$TAG
rocprofv3 -L > gpurun_out/$TAG/counters_list.txt 2>&1 || true
run() {  # name, counters
  timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv --pmc $2 -d gpurun_out/$TAG/$1 -o p -- python3 tools/prof_verify.py ${PROF_ARGS} > gpurun_out/$TAG/$1.log 2>&1
}
run sq1 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU" || exit $?
run sq2 "SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH" || exit $?
run fetch "FETCH_SIZE" || exit $?
run write "WRITE_SIZE" || exit $?
run tcc "TCC_HIT_sum TCC_MISS_sum" || exit $?
echo done
