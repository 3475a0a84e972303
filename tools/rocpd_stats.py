#!/usr/bin/env python3
"""Kernel statistics (rocprofv3 --stats layout) from a rocprofv3 results
database (ROCm 7 writes SQLite by default): Name, Calls, TotalDurationNs,
AverageNs, Percentage, MinNs, MaxNs, StdDev.  Usage: rocpd_stats.py in.db out.csv"""
import csv
import math
import sqlite3
import sys
from collections import defaultdict

db, out = sys.argv[1], sys.argv[2]
c = sqlite3.connect(db)
rows = c.execute("SELECT name, (end - start) FROM kernels").fetchall()
d = defaultdict(list)
for name, dur in rows:
    d[name].append(dur)
total = sum(sum(v) for v in d.values()) or 1
with open(out, "w", newline="") as f:
    w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
    for name, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        avg = sum(v) / len(v)
        sd = math.sqrt(sum((x - avg) ** 2 for x in v) / len(v))
        w.writerow([name, len(v), sum(v), avg, 100.0 * sum(v) / total, min(v), max(v), sd])
