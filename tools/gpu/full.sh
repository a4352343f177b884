#!/bin/bash
# Round-record session: tests, default bench (+cpu baseline), rlc bench,
# rocprofv3 kernel-trace stats of the default bench, FETCH/WRITE PMC passes.
export TMPDIR=/tmp
TAG=${TAG:-full}
D=gpurun_out/$TAG
mkdir -p $D
timeout -k 10 900 python -m pytest tests -x -q -m gpu > $D/pytest.log 2>&1
rc=$?; tail -2 $D/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python bench.py > $D/bench.json 2> $D/bench.err || exit $?
cat $D/bench.json
timeout -k 10 600 python bench.py --mode rlc --no-cpu-baseline > $D/bench_rlc.json 2> $D/bench_rlc.err || exit $?
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o bench -- python3 bench.py --no-cpu-baseline > $D/prof.log 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv --pmc $c -d $D/pmc_$c -o p -- python3 tools/prof_verify.py --rounds 131072 --iters 1 > $D/pmc_$c.log 2>&1 || exit $?
done
python3 tools/traffic_summary.py $D 131072 $D/traffic.json
