"""Summarize hipcc -Rpass-analysis=kernel-resource-usage remarks per kernel.

usage: hipcc ... -Rpass-analysis=kernel-resource-usage 2> ru.txt; python tools/resource_usage.py ru.txt
"""
import re
import sys

KEYS = {"VGPRs": "vgpr", "ScratchSize [bytes/lane]": "scratch", "Occupancy [waves/SIMD]": "occ",
        "VGPRs Spill": "vspill", "LDS Size [bytes/block]": "lds"}


def parse(path):
    rows, cur = {}, None
    for line in open(path):
        m = re.search(r"remark:\s+(Function Name|VGPRs Spill|VGPRs|ScratchSize \[bytes/lane\]|"
                      r"Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)", line)
        if not m:
            continue
        k, v = m.groups()
        if k == "Function Name":
            cur = v
            rows[cur] = {}
        elif cur:
            rows[cur][KEYS[k]] = v
    return rows


if __name__ == "__main__":
    for f, r in parse(sys.argv[1]).items():
        print(f"{f[:58]:58s} vgpr={r.get('vgpr'):>4} spill={r.get('vspill'):>5} scratch={r.get('scratch'):>5} "
              f"occ={r.get('occ')} lds={r.get('lds')}")
