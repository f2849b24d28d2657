#!/usr/bin/env python3
"""Attention section of mixed steps, from a rocprofv3 --kernel-trace output dir.

In a mixed step the decode attention (main stream) and the prefill attention (side stream)
of a layer run concurrently. For every decode-attention dispatch that overlaps a prefill
dispatch, report the decode kernel's own duration, the prefill kernel's duration and the
wall time of their union; and, for decode dispatches with no prefill beside them, the decode
duration alone. The difference "union - decode alone (same batch)" is what prefill attention
costs a mixed step.
Usage: attn_overlap.py <rocprof output dir>
"""
import csv
import glob
import json
import statistics
import sys


def main(d):
    rows = []
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                try:
                    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
                except (KeyError, ValueError):
                    pass
    rows.sort()
    dec = [r for r in rows if "decode_attn" in r[2] and "combine" not in r[2]]
    pre = [r for r in rows if "prefill_attn" in r[2]]
    # steady state: last 60% of the trace
    if not dec:
        print(json.dumps({"error": "no decode attention dispatches"}))
        return
    lo = rows[0][0] + int(0.4 * (rows[-1][1] - rows[0][0]))
    dec = [r for r in dec if r[0] >= lo]
    pre = [r for r in pre if r[0] >= lo]
    j = 0
    mixed, alone, pre_d, pre_names = [], [], [], {}
    for s, e, n in dec:
        while j < len(pre) and pre[j][1] < s - 2_000_000:
            j += 1
        ov = [p for p in pre[j:j + 8] if p[0] < e + 50_000 and p[1] > s - 50_000]
        if ov:
            us, ue = min([s] + [p[0] for p in ov]), max([e] + [p[1] for p in ov])
            mixed.append(((e - s) / 1e3, (ue - us) / 1e3, max((p[1] - p[0]) / 1e3 for p in ov)))
            for p in ov:
                pre_d.append((p[1] - p[0]) / 1e3)
                k = p[2].split("(")[0][:60]
                pre_names[k] = pre_names.get(k, 0) + 1
        else:
            alone.append((e - s) / 1e3)

    def med(x):
        return round(statistics.median(x), 2) if x else None

    print(json.dumps({
        "decode_dispatches": len(dec), "with_prefill_beside": len(mixed), "alone": len(alone),
        "decode_us_in_mixed": med([m[0] for m in mixed]), "union_us_in_mixed": med([m[1] for m in mixed]),
        "prefill_us": med(pre_d), "decode_us_alone": med(alone),
        "union_minus_decode_us": med([m[1] - m[0] for m in mixed]),
        "prefill_kernels": pre_names,
        # by the size of the prefill beside it (its kernel time): the few large prefills of
        # full mixed steps are hidden in the median above
        "by_prefill_us": {
            name: {"n": len(b), "decode_us": med([m[0] for m in b]), "union_us": med([m[1] for m in b]),
                   "union_minus_decode_us": med([m[1] - m[0] for m in b]),
                   "union_minus_decode_total_ms": round(sum(m[1] - m[0] for m in b) / 1e3, 2)}
            for name, lo_, hi_ in (("lt20", 0, 20), ("20_60", 20, 60), ("60_150", 60, 150), ("ge150", 150, 1e9))
            for b in [[m for m in mixed if lo_ <= m[2] < hi_]] if b},
    }))


if __name__ == "__main__":
    main(sys.argv[1])
