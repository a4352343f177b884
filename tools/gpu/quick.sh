#!/bin/bash
# quick iteration: gpu tests, 1M bench (no cpu baseline), one PMC pass on the verify pipeline
export TMPDIR=/tmp
TAG=${TAG:-quick}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/$TAG/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/$TAG/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || exit $?
cat gpurun_out/$TAG/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY -d gpurun_out/$TAG/sq1 -o p -- python3 tools/prof_verify.py --rounds 131072 --iters 1 > gpurun_out/$TAG/sq1.log 2>&1 || exit $?
python3 tools/pmc_summary.py gpurun_out/$TAG
