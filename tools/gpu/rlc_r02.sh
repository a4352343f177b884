#!/bin/bash
# RLC mode (configs[2]) at 1M and 10M rounds, 0.1% and 0% corruption.
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r02e}; mkdir -p $O
for n in 1000000 10000000; do
  for r in 0.001 0; do
    timeout -k 10 300 python -u bench.py --mode rlc --rounds $n --corrupt-rate $r --steps 3 --no-cpu-baseline --no-e2e > $O/rlc_${n}_${r}.json 2> $O/rlc_${n}_${r}.err || exit $?
    echo "rlc $n $r done"
  done
done
