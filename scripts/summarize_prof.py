#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats output dir into a small text table."""
import csv
import glob
import sys

d = sys.argv[1]
rows = []
for f in glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            rows.append(r)
rows.sort(key=lambda r: -float(r.get("TotalDurationNs", 0)))
tot = sum(float(r.get("TotalDurationNs", 0)) for r in rows) or 1.0
print(f"{'share':>6} {'total_ms':>10} {'calls':>7} {'avg_us':>9}  kernel")
for r in rows[:40]:
    t = float(r["TotalDurationNs"])
    print(f"{100*t/tot:6.2f} {t/1e6:10.3f} {int(r['Calls']):7d} {float(r['AverageNs'])/1e3:9.2f}  {r['Name'][:150]}")
print(f"total kernel time {tot/1e6:.3f} ms")
