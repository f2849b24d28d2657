#!/usr/bin/env python3
"""Kernel-to-kernel gaps inside the decode step's graph replays (rocprofv3 kernel trace of
benchmarks/decode_step.py): over the last half of the trace, the GPU's busy share, the gap
distribution between consecutive kernels, and the total gap time by the kernel pair around it."""
import collections
import csv
import glob
import sys


def main(d):
    ks = []
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:60]))
    ks.sort()
    if not ks:
        print("no kernels")
        return
    t0, t1 = ks[0][0], max(e for _, e, _ in ks)
    ks = [k for k in ks if k[0] >= t0 + (t1 - t0) / 2]
    span = ks[-1][1] - ks[0][0]
    busy = 0
    end = ks[0][0]
    gaps = []
    pairs = collections.Counter()
    pair_n = collections.Counter()
    for i, (s, e, n) in enumerate(ks):
        if s > end:
            if i:
                g = s - end
                gaps.append(g)
                key = (ks[i - 1][2], n)
                pairs[key] += g
                pair_n[key] += 1
        busy += max(0, e - max(s, end))
        end = max(end, e)
    gaps.sort()
    q = lambda p: gaps[min(len(gaps) - 1, int(p * len(gaps)))] / 1e3 if gaps else 0.0  # noqa: E731
    print(f"kernels {len(ks)}  span {span/1e6:.2f} ms  busy {100*busy/span:.1f}%  gaps {len(gaps)} total {sum(gaps)/1e6:.2f} ms")
    print(f"gap us: p10 {q(.1):.2f}  p50 {q(.5):.2f}  p90 {q(.9):.2f}  p99 {q(.99):.2f}  max {gaps[-1]/1e3 if gaps else 0:.2f}")
    print("total gap ms by (previous kernel -> next kernel):")
    for (a, b), g in pairs.most_common(15):
        print(f"  {g/1e6:8.2f} ms  {pair_n[(a, b)]:6d}x  avg {g/pair_n[(a, b)]/1e3:6.2f} us  {a} -> {b}")


if __name__ == "__main__":
    main(sys.argv[1])
