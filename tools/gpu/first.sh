#!/bin/bash
# GPU session script: parity tests, then a short bench (stops after any crash/timeout).
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --rounds ${BENCH_ROUNDS:-16384} --steps 2 --warmup 1 --cpu-seconds 5 > gpurun_out/bench_small.json 2> gpurun_out/bench_small.err
rc=$?
cat gpurun_out/bench_small.json; tail -5 gpurun_out/bench_small.err
exit $rc
