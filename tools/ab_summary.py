#!/usr/bin/env python3
"""Summarize A/B bench lines written by tools/gpu/session.sh ab (ab_<name>.json):
rounds/s and the engine/hash stage times per variant and repetition.

    python tools/ab_summary.py gpurun_out/<tag>
"""
import glob
import json
import os
import sys


def main(d):
    for f in sorted(glob.glob(os.path.join(d, "ab_*.json"))):
        try:
            x = json.load(open(f))
        except ValueError:
            print(os.path.basename(f), "unreadable")
            continue
        st = {k: round(v, 1) for k, v in x["stage_ms"].items() if k.startswith(("eng", "hash"))}
        fe = sum(v for k, v in x["stage_ms"].items() if k.startswith("eng_fe"))
        print(f"{os.path.basename(f):24s} {x['value']:12.0f} mism={x['verdict_mismatches']} fe_total={fe:7.1f} {st}")


if __name__ == "__main__":
    main(sys.argv[1])
