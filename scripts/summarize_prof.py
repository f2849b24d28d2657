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

    # idle gaps in the steady-state window, attributed to the kernel pair around them
    names = []
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                try:
                    names.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
                except (KeyError, ValueError):
                    pass
    names.sort()
    lo = t0 + int(0.6 * (t1 - t0))
    short = lambda n: n.split("(")[0].replace("void ", "")[:48]  # noqa: E731
    gaps, last_e, last_n = {}, None, None
    for s0, e0, n in names:
        if e0 <= lo:
            continue
        if last_e is not None and s0 - last_e > 10_000:       # > 10 us idle
            k = (short(last_n), short(n))
            g = gaps.setdefault(k, [0, 0])
            g[0] += 1
            g[1] += s0 - last_e
        if last_e is None or e0 > last_e:
            last_e, last_n = e0, n
    tot_gap = sum(v[1] for v in gaps.values())
    print(f"idle gaps > 10 us in the last 40%: {tot_gap / 1e6:.1f} ms "
          f"({100 * tot_gap / max(1, t1 - lo):.1f}% of the window)")
    for (a, b), (c, t) in sorted(gaps.items(), key=lambda kv: -kv[1][1])[:12]:
        print(f"  {t / 1e6:8.2f} ms {c:6d}x  after {a}  before {b}")

    # context of a few individual large gaps (kernel, queue, duration, gap before it)
    rows2 = []
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                try:
                    rows2.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                                  r.get("Queue_Id", "?"), r.get("Stream_Id", "?")))
                except (KeyError, ValueError):
                    pass
    rows2.sort()
    rows2 = [x for x in rows2 if x[1] > lo]
    big, ends = [], rows2[0][1] if rows2 else 0
    for i in range(1, len(rows2)):
        if rows2[i][0] - ends > 150_000:
            big.append(i)
        ends = max(ends, rows2[i][1])
    print(f"gaps > 150 us in the window: {len(big)}")
    for i in big[len(big) // 2: len(big) // 2 + 3]:
        print("  ---")
        for j in range(max(0, i - 6), min(len(rows2), i + 4)):
            s0, e0, n, q, st = rows2[j]
            print(f"  t={(s0 - rows2[i][0]) / 1e3:10.1f}us dur={(e0 - s0) / 1e3:8.1f}us q={q} s={st} {n}")
