#!/usr/bin/env python3
"""Kernel statistics (the rocprofv3 --stats summary) from a rocpd SQLite
database written by `rocprofv3 --kernel-trace` (default output format):

    python tools/rocpd_stats.py gpurun_out/<tag>/prof/bench_results.db > profiles/<round>_kernel_stats.csv
"""
import sqlite3
import sys


def main(path):
    c = sqlite3.connect(path)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name}, count(*), sum(end - start), avg(end - start), min(end - start), "
                     f"max(end - start) from kernels group by {name} order by sum(end - start) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    print('"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs"')
    for n, k, s, a, lo, hi in rows:
        print(f'"{n}",{k},{s},{a:.1f},{100.0 * s / total:.4f},{lo},{hi}')


if __name__ == "__main__":
    main(sys.argv[1])
