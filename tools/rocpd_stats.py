#!/usr/bin/env python3
"""Kernel statistics (rocprofv3 --stats layout) from a rocprofv3 rocpd SQLite database.

  python3 tools/rocpd_stats.py gpurun_out/prof/run_results.db > profiles/rNN/kernel_stats.csv
"""
import csv
import sqlite3
import statistics
import sys
from collections import defaultdict


def main():
    db = sqlite3.connect(sys.argv[1])
    dur = defaultdict(list)
    for name, d in db.execute("select name, duration from kernels"):
        dur[name].append(float(d))
    total = sum(sum(v) for v in dur.values())
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
    for name, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([name, len(v), int(sum(v)), sum(v) / len(v), 100.0 * sum(v) / total, int(min(v)),
                    int(max(v)), statistics.pstdev(v)])


if __name__ == "__main__":
    main()
