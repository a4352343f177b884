#!/bin/bash
# Engine iteration: GPU parity suite, 1M per-round bench, rocprofv3 kernel stats of the bench.
export TMPDIR=/tmp
TAG=${TAG:-eng}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/$TAG/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || exit $?
cat gpurun_out/$TAG/bench.json
if [ -n "$NO_PROF" ]; then exit 0; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof -o bench -- python3 bench.py --no-cpu-baseline --steps 2 ${BENCH_ARGS} > gpurun_out/$TAG/prof.out 2>&1 || exit $?
find gpurun_out/$TAG/prof -name "*kernel_stats*" -exec head -12 {} \;
