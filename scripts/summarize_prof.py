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

# GPU busy fraction from the kernel trace: union of kernel intervals over the analysis window.
# The window is bench.py's timed region when the trace holds its marker kernels
# (region_begin_marker_kernel ... region_end_marker_kernel, ops.region_marker), else the last
# 40% of the traced span (the steady-state part of a short run).
rows2 = []
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            try:
                rows2.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                              r.get("Queue_Id", "?"), r.get("Stream_Id", "?")))
            except (KeyError, ValueError):
                pass
if rows2:
    rows2.sort()
    t0 = rows2[0][0]
    t1 = max(e for _, e, *_ in rows2)
    begins = [e for s0, e, n, *_ in rows2 if "region_begin_marker" in n]
    ends = [s0 for s0, e, n, *_ in rows2 if "region_end_marker" in n]
    if begins and ends and max(ends) > begins[-1]:
        lo, hi = begins[-1], min(x for x in ends if x > begins[-1])
        label = "timed window (bench.py markers)"
    else:
        lo, hi = t0 + int(0.6 * (t1 - t0)), t1
        label = "last 40% of the trace (no markers)"

    def busy(lo, hi):
        tot_b, cur_s, cur_e = 0, None, None
        for s0, e0, n, *_ in rows2:
            if e0 <= lo or s0 >= hi or "region_" in n:
                continue
            s0, e0 = max(s0, lo), min(e0, hi)
            if cur_e is None or s0 > cur_e:
                if cur_e is not None:
                    tot_b += cur_e - cur_s
                cur_s, cur_e = s0, e0
            else:
                cur_e = max(cur_e, e0)
        if cur_e is not None:
            tot_b += cur_e - cur_s
        return tot_b / max(1, hi - lo)

    print(f"gpu busy {100 * busy(t0, t1):.2f}% of {(t1 - t0) / 1e9:.2f}s traced; "
          f"{label}: {100 * busy(lo, hi):.2f}% of {(hi - lo) / 1e9:.2f}s")

    # idle gaps in the window, attributed to the kernel pair around them
    short = lambda n: n.split("(")[0].replace("void ", "")[:48]  # noqa: E731
    win = [x for x in rows2 if x[1] > lo and x[0] < hi and "region_" not in x[2]]
    gaps, last_e, last_n = {}, lo, "<window start>"
    hist = {"10-50us": [0, 0], "50-200us": [0, 0], "0.2-1ms": [0, 0], ">1ms": [0, 0]}
    for s0, e0, n, *_ in win + [(hi, hi, "<window end>", "", "")]:
        g = s0 - last_e
        if g > 10_000:       # > 10 us idle
            k = (short(last_n), short(n))
            v = gaps.setdefault(k, [0, 0])
            v[0] += 1
            v[1] += g
            b = "10-50us" if g < 50_000 else "50-200us" if g < 200_000 else "0.2-1ms" if g < 1_000_000 else ">1ms"
            hist[b][0] += 1
            hist[b][1] += g
        if e0 > last_e:
            last_e, last_n = e0, n
    tot_gap = sum(v[1] for v in gaps.values())
    print(f"idle gaps > 10 us in the window: {tot_gap / 1e6:.1f} ms "
          f"({100 * tot_gap / max(1, hi - lo):.2f}% of the window)")
    print("  by length: " + ", ".join(f"{k}: {c} gaps {t / 1e6:.1f} ms" for k, (c, t) in hist.items()))
    for (a, b), (c, t) in sorted(gaps.items(), key=lambda kv: -kv[1][1])[:12]:
        print(f"  {t / 1e6:8.2f} ms {c:6d}x  after {a}  before {b}")

    # context of a few individual large gaps (kernel, queue, duration, gap before it)
    big, ends_ = [], win[0][1] if win else 0
    for i in range(1, len(win)):
        if win[i][0] - ends_ > 150_000:
            big.append(i)
        ends_ = max(ends_, win[i][1])
    print(f"gaps > 150 us in the window: {len(big)}")
    for i in big[len(big) // 2: len(big) // 2 + 3]:
        print("  ---")
        for j in range(max(0, i - 6), min(len(win), i + 4)):
            s0, e0, n, q, st = win[j]
            print(f"  t={(s0 - win[i][0]) / 1e3:10.1f}us dur={(e0 - s0) / 1e3:8.1f}us q={q} s={st} {short(n)}")
