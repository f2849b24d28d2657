#!/usr/bin/env python3
"""Row-split A/B for the N = 4,096 projection GEMMs (o and down of Llama-3-8B) at the token
counts of full mixed steps: a 4,096-token prefill budget plus up to 256 decode rows makes
M = 4,352, where 256 x 256 output tiles come to 17 x 16 = 272 — one full wave of 256 CUs and
a second wave of 16 tiles. Splitting the rows as 4,096 + (M - 4,096) runs the big part as
exactly one wave and the remainder right after it on the same (MALL-warm) weights.

Weights rotate over 32 layer copies per GEMM, as in a forward pass (cold in the caches).
Prints one JSON line per (GEMM, M): microseconds per call fused vs split."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="4160,4352,4608,8448")
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--only", default="", help="comma-separated GEMM names")
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--splits", default="4096",
                    help="comma-separated split rules: an int (rows), or mN (M rounded down to a multiple of N), "
                         "or -N (M - N)")
    a = ap.parse_args()
    from nv_genai_amd import ops
    from nv_genai_amd.ops.gemm_tuning import use_tuned_gemms

    print(json.dumps({"table_loaded": use_tuned_gemms()}), flush=True)
    dev = torch.device("cuda")
    shapes = {"o": (4096, 4096), "down": (4096, 14336), "qkv": (6144, 4096), "gate_up": (28672, 4096)}
    for name, (N, K) in shapes.items():
        if a.only and name not in a.only.split(","):
            continue
        Ws = [torch.empty(N, K, device=dev, dtype=torch.bfloat16).uniform_(-0.05, 0.05) for _ in range(a.layers)]
        for m in [int(x) for x in a.ms.split(",")]:
            x = torch.empty(m, K, device=dev, dtype=torch.bfloat16).uniform_(-1, 1)
            out = torch.empty(m, N, device=dev, dtype=torch.bfloat16)
            res = {"gemm": name, "M": m}
            def rule(r):
                if r.startswith("m"):
                    return m // int(r[1:]) * int(r[1:])
                if r.startswith("-"):
                    return m - int(r[1:])
                return int(r)
            variants = [("fused", 0)] + [(f"split_{r}", rule(r)) for r in a.splits.split(",")]
            variants = [(t, sp) for t, sp in variants if t == "fused" or 0 < sp < m]
            for tag, split in variants:
                def run():
                    for w in Ws:
                        ops.linear_rows_split(x, w, out, split)
                for _ in range(2):
                    run()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    run()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / (a.iters * len(Ws))
                res[tag] = {"us": round(us, 1), "PF": round(2.0 * m * N * K / us / 1e9, 3)}
            best = min(res[t]["us"] for t, _ in variants)
            res["best"] = next(t for t, _ in variants if res[t]["us"] == best)
            print(json.dumps(res), flush=True)
        del Ws


if __name__ == "__main__":
    main()
