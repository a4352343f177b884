#!/bin/bash
# Round-4 session x: throughput against batch size on the final build --
# per-round and RLC (0.1% corrupted) verify of chained chains of 4Ki, 64Ki,
# 512Ki and 2Mi rounds (one bench.py run each, HBM-resident records).
export TMPDIR=/tmp
O=gpurun_out/r04x
mkdir -p $O
for n in 4096 65536 524288 2097152; do
  echo "== n=$n $(date +%T)"
  timeout -k 10 300 python -u bench.py --rounds $n --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-legs > $O/bench_$n.json 2> $O/bench_$n.err || exit $?
done
echo done
