#!/bin/bash
# GPU session: parity tests, full-size bench, rocprofv3 kernel-trace stats of the same bench.
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r01}
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
tail -4 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python bench.py ${BENCH_ARGS} > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err
rc=$?
cat gpurun_out/bench_${TAG}.json; tail -3 gpurun_out/bench_${TAG}.err
if [ $rc -ne 0 ]; then exit $rc; fi
if [ -n "$NO_PROF" ]; then exit 0; fi
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o bench -- python3 bench.py ${BENCH_ARGS} --no-cpu-baseline > gpurun_out/prof_${TAG}.out 2>&1
rc=$?
tail -3 gpurun_out/prof_${TAG}.out
find gpurun_out/prof_${TAG} -name "*stats*" | head
exit $rc
