"""Sweep the decode-shape projection GEMM (csrc/kernels/gemm_skinny.hip) over its tile
configurations and K splits for the Llama-3-8B projections at small M, against the tuned
library GEMM, with weights rotating over enough copies to miss the 256 MB MALL (a decode step
streams 32 layers of weights, so no layer's weights are cache-warm).

Per (shape, M): the library time, then every (cfg, split) that makes a sensible grid:
``gemm`` = the skinny kernel alone (bf16 out for split 1 / SwiGLU, fp32 slabs otherwise),
``total`` = gemm + a standalone split-K reduce (the engine folds the reduce into the consumer
kernel, so the truth lies between the two). One JSON line per shape and M with the best.
"""
import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from nv_genai_amd import ops  # noqa: E402
from nv_genai_amd.ops.gemm_tuning import use_tuned_gemms  # noqa: E402

SHAPES = {"qkv": (6144, 4096, 0), "o": (4096, 4096, 0), "gate_up": (28672, 4096, 2),
          "down": (4096, 14336, 0), "lm_head": (128256, 4096, 0)}


def timeit(fn, n_rot, iters):
    for i in range(3):
        fn(i % n_rot)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(iters):
        fn(i % n_rot)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3   # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="64,128,256,512")
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--krot", type=int, default=0)
    ap.add_argument("--wpack", action="store_true", help="tile-packed weights (ops.pack_weight)")
    ap.add_argument("--xpack", action="store_true", help="tile-packed activations (ops.pack_rows)")
    ap.add_argument("--cfgs", default=None, help="comma list (default: all)")
    ap.add_argument("--check", action="store_true", help="numerics of the best config vs fp32")
    ap.add_argument("--all", action="store_true", help="print every (cfg, split) result")
    ap.add_argument("--rot-mb", type=float, default=640.0,
                    help="rotate weight copies totalling at least this many MB (640: past the 256 MB MALL; 0: one copy, cache-warm)")
    a = ap.parse_args()
    print("tuned table:", use_tuned_gemms(), flush=True)
    C = ops.kernels()
    ncfg = C.skinny_cfg_count()
    cfgs = [int(c) for c in a.cfgs.split(",")] if a.cfgs else list(range(ncfg))
    info = {c: C.skinny_cfg(c) for c in cfgs}
    dev = torch.device("cuda")
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    for name in a.shapes.split(","):
        N, K, epi_full = SHAPES[name]
        wbytes = N * K * 2
        n_rot = max(2, math.ceil(a.rot_mb * 1e6 / wbytes)) if a.rot_mb > 0 else 1
        Ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16, generator=g) * 0.02 for _ in range(n_rot)]
        for M in [int(m) for m in a.ms.split(",")]:
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16, generator=g)
            Nout = N // 2 if epi_full == 2 else N
            if epi_full == 2:
                lib_us = timeit(lambda i: ops.silu_mul(x @ Ws[i].t()), n_rot, a.iters)
            else:
                lib_us = timeit(lambda i: x @ Ws[i].t(), n_rot, a.iters)
            res = []
            packed = {}
            for c in cfgs:
                BN, BM, WN, WM, NS = info[c]
                nn = (Nout // (BN // 2)) if epi_full == 2 else -(-N // BN)
                if epi_full == 2 and Nout % (BN // 2):
                    continue
                nm = -(-M // BM)
                if BM > 2 * M and BM > 32:   # mostly padding rows
                    continue
                splits = [1] if epi_full == 2 else [s for s in (1, 2, 3, 4, 6, 8, 12, 16) if s <= K // 64]
                for s in splits:
                    blocks = nn * nm * s
                    if blocks < 32 or blocks > 4096 or (s > 1 and nn * nm >= 512):
                        continue
                    epi = epi_full if s == 1 else 1
                    out = (torch.empty(s, M, N, dtype=torch.float32, device=dev) if epi == 1
                           else torch.empty(M, Nout, dtype=torch.bfloat16, device=dev))
                    red = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
                    if a.wpack:
                        key = (BN, epi_full)
                        if key not in packed:
                            packed[key] = [ops.pack_weight(w, BN, epi_full) for w in Ws]
                        Wu, pk, nout = packed[key], 1, Nout
                    else:
                        Wu, pk, nout = Ws, 0, 0
                    if a.xpack:
                        xu, xm = ops.pack_rows(x, BM), M
                    else:
                        xu, xm = x, 0
                    t_g = timeit(lambda i: C.skinny_gemm(out, xu, Wu[i], epi, s, c, a.krot, pk, nout, xm, K), n_rot, a.iters)
                    if epi == 1:
                        t_t = timeit(lambda i: (C.skinny_gemm(out, xu, Wu[i], epi, s, c, a.krot, pk, nout, xm, K),
                                                C.splitk_reduce(red, out, s)), n_rot, a.iters)
                    else:
                        t_t = t_g
                    r = {"cfg": c, "tile": [BN, BM, WN, WM, NS], "split": s, "blocks": blocks,
                         "gemm_us": round(t_g, 2), "total_us": round(t_t, 2)}
                    res.append(r)
                    if a.all:
                        print(json.dumps({"shape": name, "M": M, **r}), flush=True)
            best = min(res, key=lambda r: r["gemm_us"]) if res else None
            best_t = min(res, key=lambda r: r["total_us"]) if res else None
            row = {"shape": name, "M": M, "N": N, "K": K, "lib_us": round(lib_us, 2),
                   "lib_TBps": round(wbytes / lib_us / 1e6, 2), "best_gemm": best, "best_total": best_t}
            if best:
                row["best_TBps"] = round(wbytes / best["gemm_us"] / 1e6, 2)
                row["speedup_gemm"] = round(lib_us / best["gemm_us"], 2)
                row["speedup_total"] = round(lib_us / best_t["total_us"], 2)
            if a.check and best:
                c, s = best["cfg"], best["split"]
                w = Ws[0]
                epi = epi_full if s == 1 else 1
                BN = info[c][0]
                y = (ops.skinny_gemm(x, ops.pack_weight(w, BN, epi_full), c, s, epi, krot=a.krot, n_out=Nout)
                     if a.wpack else ops.skinny_gemm(x, w, c, s, epi, krot=a.krot))
                if epi == 1:
                    y = y.sum(0)
                refm = x.float() @ w.float().t()
                if epi_full == 2:
                    refm = torch.nn.functional.silu(refm[:, :Nout]) * refm[:, Nout:]
                err = ((y.float() - refm).norm(dim=1) / refm.norm(dim=1).clamp_min(1e-6)).max().item()
                row["max_row_rel_err"] = float(f"{err:.3e}")
            print(json.dumps(row), flush=True)
            del packed
        del Ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
