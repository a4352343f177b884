#!/bin/bash
# HBM traffic of the per-round pipeline: two PMC passes (FETCH_SIZE and
# WRITE_SIZE cannot share a pass), kernel-trace only, one 131072-round engine
# chunk.  Summarized (with the line-buffer calibration) by tools/traffic_summary.py.
export TMPDIR=/tmp
TAG=${TAG:-traffic}
O=gpurun_out/$TAG
mkdir -p $O
run() {  # name, counters
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $2 -d $O/$1 -o p -- python3 tools/prof_verify.py --rounds 131072 --iters 1 > $O/$1.log 2>&1
}
run fetch "FETCH_SIZE" || exit $?
run write "WRITE_SIZE" || exit $?
python3 tools/traffic_summary.py $O 131072 $O/traffic.json
