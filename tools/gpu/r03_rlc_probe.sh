#!/bin/bash
# RLC (bucket-MSM root) tests + benches at 0% / 0.1% corruption, then the
# fused lines+Miller occupancy probe A/B on the per-round path.
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03f}
mkdir -p $O
TAG=${TAG:-r03f} PYTEST_K="rlc or multi or parity" NOBENCH=1 tools/gpu/r03_session.sh || exit $?
for cr in 0 0.001; do
  timeout -k 10 300 python -u bench.py --mode rlc --corrupt-rate $cr --no-legs --no-cpu-baseline --no-e2e --no-ingest --steps 3 > $O/rlc_$cr.json 2>> $O/rlc.err || exit 1
done
for probe in 0 1 0 1; do
  DGPU_ENG_FUSED_PROBE=$probe timeout -k 10 300 python -u bench.py --no-legs --no-rlc --no-cpu-baseline --no-e2e --no-ingest --steps 2 --warmup 1 --rounds 2000000 > $O/probe_$probe.json.tmp 2>> $O/probe.err || exit 1
  cat $O/probe_$probe.json.tmp >> $O/probe_$probe.jsonl
done
echo done
