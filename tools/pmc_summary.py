"""Aggregate rocprofv3 --pmc CSV passes (tools/gpu/pmc.sh) per kernel."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d):
    vals = defaultdict(lambda: defaultdict(float))
    durs = {}
    for f in glob.glob(os.path.join(d, "*", "p_counter_collection.csv")):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = r["Kernel_Name"].split("(")[0]
                vals[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for f in glob.glob(os.path.join(d, "*", "p_kernel_trace.csv")):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = r["Kernel_Name"].split("(")[0]
                durs.setdefault(k, []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for k, v in vals.items():
        print(k)
        dd = durs.get(k)
        if dd:
            print(f"   duration_ns(median over passes) {sorted(dd)[len(dd)//2]}")
        for c in sorted(v):
            print(f"   {c:24s} {v[c]:.4g}")


if __name__ == "__main__":
    main(sys.argv[1])
