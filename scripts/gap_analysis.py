#!/usr/bin/env python3
"""GPU idle-gap analysis of a rocprofv3 kernel trace: over the last ``--tail`` fraction of the
trace (steady state), list the idle gaps between consecutive kernels by size, with the
kernels on either side, and the gap histogram. With ``--marker-trace`` output present, each
big gap is also tagged with the ROCTx range (engine step) active on the host at its start."""
import argparse
import collections
import csv
import glob


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--tail", type=float, default=0.4)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    ks = []
    for f in glob.glob(f"{a.dir}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:70]))
    ks.sort()
    if not ks:
        print("no kernels")
        return
    t0, t1 = ks[0][0], max(e for _, e, _ in ks)
    cut = t1 - a.tail * (t1 - t0)
    ks = [k for k in ks if k[0] >= cut]
    marks = []
    print("trace files:", sorted({f.split("/")[-1] for f in glob.glob(f"{a.dir}/**/*.csv", recursive=True)}))
    for f in glob.glob(f"{a.dir}/**/*marker*.csv", recursive=True):
        rd = csv.DictReader(open(f))
        print("marker columns:", rd.fieldnames)
        for r in rd:
            try:
                name = r.get("Function") or r.get("Name") or r.get("Message") or ""
                marks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name[:60]))
            except (KeyError, ValueError, TypeError):
                pass
    marks.sort()
    apis = []
    for f in glob.glob(f"{a.dir}/**/*hip_api_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            try:
                apis.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Function", "")[:40]))
            except (KeyError, ValueError, TypeError):
                pass
    apis.sort()
    gaps, end = [], ks[0][1]
    prev = ks[0][2]
    for j, (s, e, n) in enumerate(ks[1:], start=1):
        if s > end:
            nxt = " | ".join(k[2][:28] for k in ks[j:j + 4])
            gaps.append((s - end, end, prev, nxt))
        if e > end:
            end, prev = e, n
    span = ks[-1][1] - ks[0][0]
    tot = sum(g for g, *_ in gaps)
    print(f"steady-state span {span / 1e6:.1f} ms, idle {tot / 1e6:.2f} ms ({100 * tot / span:.1f}%), {len(gaps)} gaps")
    hist = collections.Counter()
    for g, *_ in gaps:
        b = "<5us" if g < 5e3 else "<20us" if g < 2e4 else "<100us" if g < 1e5 else "<1ms" if g < 1e6 else ">=1ms"
        hist[b] += g
    for b in ("<5us", "<20us", "<100us", "<1ms", ">=1ms"):
        print(f"  gaps {b:>7}: {hist[b] / 1e6:8.2f} ms")
    print("largest gaps:")
    for g, at, p, n in sorted(gaps, reverse=True)[: a.top]:
        m = [x[2] for x in marks if x[0] <= at <= x[1]]
        hm = [x for x in marks if x[0] <= at + g and x[1] >= at]
        desc = ""
        if hm:
            b, e, nm = hm[-1]
            desc = f"{nm!r} range {(e - b) / 1e3:.0f} us, gap starts {(at - b) / 1e3:+.0f} us into it"
        print(f"  {g / 1e3:9.1f} us  after {p[:30]!r} then {n[:60]}  host: {desc}")
        # HIP API calls in flight or issued during the gap (long ones = the host blocked)
        ov = [(e - b, nm, (b - at) / 1e3) for b, e, nm in apis if b <= at + g and e >= at and e - b > 200e3]
        for d, nm, off in sorted(ov, reverse=True)[:3]:
            print(f"        api {nm:40s} {d / 1e3:8.1f} us  (starts {off:+.1f} us from gap start)")


if __name__ == "__main__":
    main()
