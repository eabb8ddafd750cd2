#!/usr/bin/env python3
"""Kernel statistics from a rocprofv3 rocpd database (ROCm 7.2 writes a .db unless given
--output-format csv): the same columns as rocprofv3's kernel_stats.csv.

    python tools/rocpd_stats.py gpurun_out/prof/run_results.db > profiles/rNN_kernel_stats.csv
"""
import csv
import sqlite3
import statistics
import sys
from collections import defaultdict


def main(path):
    c = sqlite3.connect(path)
    durs = defaultdict(list)
    for name, d in c.execute("select name, duration from kernels"):
        durs[name].append(int(d))
    total = sum(sum(v) for v in durs.values()) or 1
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
    for name, v in sorted(durs.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([name, len(v), sum(v), sum(v) / len(v), round(100.0 * sum(v) / total, 2), min(v), max(v),
                    statistics.pstdev(v) if len(v) > 1 else 0.0])


if __name__ == "__main__":
    main(sys.argv[1])
