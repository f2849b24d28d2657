"""Composition of the headline's scheduler steps from bench.py --timeline-out: per step kind,
decode rows and prefill tokens; the launch-to-launch wall time by class (the pipelined loop
launches one step per GPU step, so the deltas track GPU step time)."""
import collections
import json
import sys


def main(path):
    tl = json.load(open(path))
    rows = []
    for a, b in zip(tl, tl[1:]):
        pf = a["tokens"] - a["decode_rows"]
        rows.append((a["kind"], a["decode_rows"], pf, a["tokens"], (b["t"] - a["t"]) * 1e3))
    cls = collections.defaultdict(list)
    for kind, nd, pf, tok, dt in rows:
        if kind == "decode":
            c = "decode"
        elif pf <= 16:
            c = "mixed, prefill <= 16"
        elif pf <= 256:
            c = "mixed, prefill 17-256"
        elif tok <= 2048:
            c = "mixed, <= 2048 tokens"
        else:
            c = "mixed/prefill, > 2048 tokens"
        cls[c].append((pf, dt))
    out = {}
    for c, v in sorted(cls.items()):
        dts = sorted(x[1] for x in v)
        pfs = sorted(x[0] for x in v)
        out[c] = {"steps": len(v), "prefill_tokens_median": pfs[len(pfs) // 2],
                  "prefill_tokens_total": sum(pfs), "ms_median": round(dts[len(dts) // 2], 2),
                  "ms_total": round(sum(dts), 1)}
    hist = collections.Counter(min(pf, 300) // 4 * 4 for _, _, pf, _, _ in rows if pf <= 300)
    out["prefill_chunk_hist_le300"] = dict(sorted(hist.items()))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
