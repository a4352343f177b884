"""Per-round HBM traffic of each verify kernel from separate rocprofv3 PMC
passes (FETCH_SIZE, WRITE_SIZE; tools/gpu/session.sh traffic), written to
profiles/<tag>_traffic.json for bench.py's roofline.traffic.

Passes are subdirectories of the traffic directory: `fetch` and `write` over
the shipped build, and `write_cal`, a WRITE_SIZE pass under DGPU_LINES=engine
so that k_eng_lines (the write calibrator) runs.  Since round 3 the default
build writes the line buffer from k_lines_thr, whose spill write-backs add to
its stores, so k_eng_lines is only present in that extra pass (rounds 4's
files had no calibrator and write_cal 1.0: rocprof's WRITE_SIZE unit, KB).

MI355X_MICROARCH.md: FETCH_SIZE reads 1/2 of the bytes for 16-B-per-lane
streaming loads and other access widths are uncalibrated.  The engine's own
line buffer gives an exact calibration for its 4-B-per-lane SoA accesses:
k_eng_lines stores exactly 68 x 12 x 14 x 4 = 45,696 B per round and
k_eng_miller loads exactly those bytes (inputs/constants of either kernel are
< 1% of that), so write_cal = 45,696 / WRITE_SIZE(k_eng_lines) and
fetch_cal = 45,696 / FETCH_SIZE(k_eng_miller); the corrected per-round bytes
(raw x cal) are what bench.py reports.  The line buffer (6 GB per chunk) far
exceeds the 256 MiB Infinity Cache, so these bytes do reach HBM."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

LINE_BYTES_PER_ROUND = 68 * 12 * 14 * 4


def _totals(d):
    tot = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                tot[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]] += float(r["Counter_Value"])
    return tot


def main(d, rounds, out):
    cal_dir = os.path.join(d, "write_cal")
    tot = defaultdict(lambda: defaultdict(float))
    for sub in os.listdir(d):
        if sub == "write_cal" or not os.path.isdir(os.path.join(d, sub)):
            continue
        for k, v in _totals(os.path.join(d, sub)).items():
            for c, x in v.items():
                tot[k][c] += x
    raw = {k: {"fetch": v.get("FETCH_SIZE", 0) / rounds, "write": v.get("WRITE_SIZE", 0) / rounds}
           for k, v in tot.items() if "FETCH_SIZE" in v or "WRITE_SIZE" in v}
    wl = raw.get("dgpu::k_eng_lines", {}).get("write")
    if not wl and os.path.isdir(cal_dir):
        wl = _totals(cal_dir).get("dgpu::k_eng_lines", {}).get("WRITE_SIZE", 0) / rounds or None
    fm = raw.get("dgpu::k_eng_miller", {}).get("fetch")
    write_cal = LINE_BYTES_PER_ROUND / wl if wl else 1.0
    fetch_cal = LINE_BYTES_PER_ROUND / fm if fm else 1.0
    res = {k: {"fetch_bytes_per_round": v["fetch"] * fetch_cal, "write_bytes_per_round": v["write"] * write_cal,
               "raw_fetch_size_per_round": v["fetch"], "raw_write_size_per_round": v["write"]}
           for k, v in raw.items()}
    if not wl:
        raise SystemExit("no write calibrator (k_eng_lines) in any pass: run the write_cal pass")
    doc = {"rounds": rounds, "fetch_cal": fetch_cal, "write_cal": write_cal, "kernels": res,
           "note": " ".join(__doc__.split("\n\n")[1:3])}
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps({k: v for k, v in doc.items() if k != "note"}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), sys.argv[3])
