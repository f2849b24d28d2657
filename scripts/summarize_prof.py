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

# GPU busy fraction from the kernel trace: union of kernel intervals over the traced span,
# and over the last 40% of it (the timed, steady-state part of a bench run)
iv = []
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            try:
                iv.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
            except (KeyError, ValueError):
                pass
if iv:
    iv.sort()

    def busy(lo):
        tot_b, cur_s, cur_e = 0, None, None
        for s0, e0 in iv:
            if e0 <= lo:
                continue
            s0 = max(s0, lo)
            if cur_e is None or s0 > cur_e:
                if cur_e is not None:
                    tot_b += cur_e - cur_s
                cur_s, cur_e = s0, e0
            else:
                cur_e = max(cur_e, e0)
        if cur_e is not None:
            tot_b += cur_e - cur_s
        span = max(e for _, e in iv) - lo
        return tot_b / max(1, span), span

    t0 = iv[0][0]
    t1 = max(e for _, e in iv)
    b_all, span = busy(t0)
    b_tail, tail = busy(t0 + int(0.6 * (t1 - t0)))
    print(f"gpu busy {100 * b_all:.1f}% of {span / 1e9:.2f}s traced; last 40%: {100 * b_tail:.1f}% of {tail / 1e9:.2f}s")
