"""Per-round HBM traffic of each verify kernel from separate rocprofv3 PMC
passes (FETCH_SIZE, WRITE_SIZE; tools/gpu/full.sh), written to
profiles/<tag>_traffic.json for bench.py's roofline.traffic.

FETCH_SIZE/WRITE_SIZE are taken as reported (bytes).  MI355X_MICROARCH.md:
FETCH_SIZE reads 1/2 of the bytes only for 16-B-per-lane streaming loads;
these kernels use 4-B-per-lane coalesced accesses (uncalibrated width), so no
correction factor is applied; treat the figure as indicative."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main(d, rounds, out):
    tot = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(os.path.join(d, "*", "p_counter_collection.csv")):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                tot[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]] += float(r["Counter_Value"])
    res = {}
    for k, v in tot.items():
        if "FETCH_SIZE" in v or "WRITE_SIZE" in v:
            res[k] = {"fetch_bytes_per_round": v.get("FETCH_SIZE", 0) / rounds,
                      "write_bytes_per_round": v.get("WRITE_SIZE", 0) / rounds}
    with open(out, "w") as f:
        json.dump({"rounds": rounds, "kernels": res, "note": __doc__.split("\n\n")[1]}, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), sys.argv[3])
