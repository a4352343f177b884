#!/bin/bash
# PMC counters per engine op (one rocprofv3 run per op, kernel-trace only).
export TMPDIR=/tmp
TAG=${TAG:-ebpmc}
O=gpurun_out/$TAG
mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
for op in ${OPS:-E_CYC_lin E_CYC_prod E_MUL M_SQR}; do
  ENGBENCH_ONLY=$op timeout -s KILL 60 rocprofv3 --kernel-trace --output-format csv --pmc ${PMC:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY} -d $O/$op -o p -- tools/engbench/engbench_base 64 > $O/$op.log 2>&1 || exit $?
done
echo done
