#!/usr/bin/env python3
"""Collect an A/B session's bench lines (tools/gpu/session.sh ab) and engine op
microbench lines into one record: ab_record.py DIR WHAT OUT.json"""
import glob
import json
import os
import sys

d, what, out = sys.argv[1], sys.argv[2], sys.argv[3]
runs = []
for f in sorted(glob.glob(os.path.join(d, "*_[12].json"))):
    j = json.loads(open(f).read().strip().splitlines()[-1])
    runs.append({"variant": os.path.basename(f)[:-5], "rounds_per_s": j["value"],
                 "verdict_mismatches": j["verdict_mismatches"], "stage_ms": j["stage_ms"]})
eb = {}
for f in sorted(glob.glob(os.path.join(d, "engbench_*.jsonl"))):
    eb[os.path.basename(f)[9:-6]] = [json.loads(x) for x in open(f) if x.strip()]
json.dump({"what": what, "runs": runs, "engbench": eb}, open(out, "w"), indent=1)
print(out, len(runs), "runs")
