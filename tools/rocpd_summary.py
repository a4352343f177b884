"""Summarize a rocprofv3 --kernel-trace --stats run (rocpd SQLite or CSV
output) into a per-kernel table: calls, total, average, share.

    python tools/rocpd_summary.py gpurun_out/prof_r01a > profiles/r01_rocprof_kernel_stats.txt
"""
import csv
import glob
import os
import sqlite3
import sys


def main(d):
    dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    rows = []
    if dbs:
        c = sqlite3.connect(dbs[0])
        agg = {}
        for name, dur in c.execute("select name, duration from kernels"):  # per-dispatch ns
            a = agg.setdefault(name, [0, 0.0])
            a[0] += 1
            a[1] += dur
        tot = sum(v[1] for v in agg.values()) or 1.0
        for name, (calls, total) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            rows.append((name, calls, total, total / calls, 100.0 * total / tot))
        src = os.path.relpath(dbs[0])
    else:
        cs = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
        if not cs:
            sys.exit("no rocprofv3 output under " + d)
        src = os.path.relpath(cs[0])
        with open(cs[0]) as f:
            for r in csv.DictReader(f):
                rows.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]), float(r["AverageNs"]),
                             float(r["Percentage"])))
    print(f"# rocprofv3 --kernel-trace --stats summary ({src}); durations as reported by rocprofv3 (ns)")
    print(f"{'calls':>6} {'total_ns':>16} {'avg_ns':>16} {'pct':>7}  kernel")
    for name, calls, total, avg, pct in rows:
        print(f"{calls:>6} {total:>16.1f} {avg:>16.1f} {pct:>6.2f}%  {name[:110]}")


if __name__ == "__main__":
    main(sys.argv[1])
