"""Build the decode-shape GEMM selection table (``nv_genai_amd/assets/skinny_gemm_gfx950.json``)
by timing each projection together with the kernel that consumes its output, exactly as the
model runs them, against the library path, at every decode / small-mixed row count M:

* ``qkv``  : skinny GEMM (bf16, or K-split fp32 slabs summed by the RoPE kernel) + RoPE vs
  ``x @ W^T`` + RoPE;
* ``o``, ``down`` : skinny GEMM + ``splitk_add_rmsnorm`` (the residual add + RMSNorm reading the
  slabs) vs ``x @ W^T`` + ``add_rmsnorm``;
* ``gate_up`` : skinny GEMM with the SwiGLU epilogue vs ``x @ W^T`` + ``silu_mul``;
* ``lm_head`` : skinny GEMM writing fp32 logits vs ``(x @ W^T).float()``.

Weights rotate over copies past the 256 MB MALL (a decode step streams every layer's weights
once). One JSON line per (shape, M) plus the table file: for each shape and M the winning
(cfg, split) or "lib".

Usage: ``python benchmarks/skinny_table.py --model llama3-8b [--out FILE]``.
"""
import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from nv_genai_amd import ops  # noqa: E402
from nv_genai_amd.models.config import llama_config  # noqa: E402
from nv_genai_amd.ops.gemm_tuning import use_tuned_gemms  # noqa: E402

MS = (16, 32, 64, 96, 128, 160, 192, 224, 256, 320, 384, 448, 512)


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
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--ms", default=",".join(map(str, MS)))
    ap.add_argument("--shapes", default="qkv,o,gate_up,down,lm_head")
    ap.add_argument("--iters", type=int, default=25)
    ap.add_argument("--out", default=None, help="table file (default: the shipped asset)")
    ap.add_argument("--merge", default=None, help="update this table file with the measured shapes only")
    ap.add_argument("--cfgs", default=None, help="comma list of tile configurations to try (default: all)")
    ap.add_argument("--all", action="store_true", help="also print every (cfg, split) time")
    ap.add_argument("--tp", type=int, default=1, help="per-rank shapes of a TP group of this size "
                    "(column-parallel q/k/v, gate/up, LM head; row-parallel o, down)")
    a = ap.parse_args()
    use_tuned_gemms()
    cfg = llama_config(a.model)
    H, F, D, tp = cfg.hidden, cfg.ffn // a.tp, cfg.head_dim, a.tp
    shapes = {"qkv": ((cfg.heads + 2 * cfg.kv_heads) // tp * D, H), "o": (H, cfg.heads // tp * D),
              "gate_up": (2 * F, H), "down": (H, F), "lm_head": (-(-cfg.vocab_size // tp), H)}
    C = ops.kernels()
    cfgs = [int(c) for c in a.cfgs.split(",")] if a.cfgs else list(range(C.skinny_cfg_count()))
    info = {c: C.skinny_cfg(c) for c in cfgs}
    dev = torch.device("cuda")
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    table = {}
    for name in a.shapes.split(","):
        N, K = shapes[name]
        n_rot = max(2, math.ceil(640e6 / (N * K * 2)))
        Ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16, generator=g) * 0.02 for _ in range(n_rot)]
        nw = torch.ones(N if name in ("o", "down") else 1, device=dev, dtype=torch.bfloat16)
        # qkv feeds the RoPE kernel, which sums K-split slabs itself (no cache write here)
        Hq, Hkv = cfg.heads // tp, max(1, cfg.kv_heads // tp)
        cos_sin = ops.rope_cos_sin(64, D, cfg.rope_theta).to(dev)

        def rope(q, part=None):
            pos = torch.zeros(q.shape[0], dtype=torch.int32, device=dev)
            C.rope_cache(q, pos, cos_sin, None, None, None, Hq, Hkv, D, 1.0, 1.0, part)
        entry = table.setdefault(f"{N}x{K}", {"shape": name, "by_m": {}})
        for M in [int(m) for m in a.ms.split(",")]:
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16, generator=g)
            resid = torch.randn(M, N, device=dev, dtype=torch.bfloat16, generator=g) if name in ("o", "down") else None
            normed = torch.empty_like(resid) if resid is not None else None
            if name == "gate_up":
                lib = timeit(lambda i: ops.silu_mul(x @ Ws[i].t()), n_rot, a.iters)
            elif name in ("o", "down"):
                lib = timeit(lambda i: ops.add_rmsnorm(resid, x @ Ws[i].t(), nw, 1e-5, out=normed), n_rot, a.iters)
            elif name == "lm_head":
                lib = timeit(lambda i: (x @ Ws[i].t()).float(), n_rot, a.iters)
            else:
                lib = timeit(lambda i: rope(x @ Ws[i].t()), n_rot, a.iters)
            best = None
            for c in cfgs:
                BN, BM = info[c][:2]
                if BM > 2 * M and BM > 32:
                    continue
                if name == "gate_up" and (N // 2) % (BN // 2):
                    continue
                nn = (N // 2) // (BN // 2) if name == "gate_up" else -(-N // BN)
                nm = -(-M // BM)
                splits = [1] if name == "lm_head" else [s for s in (1, 2, 3, 4, 6, 8, 12, 16) if s <= K // 64]
                if name == "gate_up":
                    splits = [s for s in splits if s <= 4]
                for s in splits:
                    blocks = nn * nm * s
                    if blocks < 16 or blocks > 4096 or (s > 1 and nn * nm >= 512):
                        continue
                    if name == "gate_up" and s > 1:   # K-split slabs summed by the SwiGLU kernel
                        out = torch.empty(s, M, N, device=dev)
                        h = torch.empty(M, N // 2, device=dev, dtype=torch.bfloat16)
                        fn = (lambda i, out=out, c=c, s=s, h=h: (C.skinny_gemm(out, x, Ws[i], 1, s, c, 0, 0, 0, 0, 0),
                                                                 C.splitk_swiglu(h, out, s)))
                    elif name == "gate_up":
                        out = torch.empty(M, N // 2, device=dev, dtype=torch.bfloat16)
                        fn = (lambda i, out=out, c=c: C.skinny_gemm(out, x, Ws[i], 2, 1, c, 0, 0, 0, 0, 0))
                    elif name == "lm_head":
                        out = torch.empty(1, M, N, device=dev)
                        fn = (lambda i, out=out, c=c: C.skinny_gemm(out, x, Ws[i], 1, 1, c, 0, 0, 0, 0, 0))
                    elif name in ("o", "down"):
                        if s == 1:
                            out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
                            fn = (lambda i, out=out, c=c: (C.skinny_gemm(out, x, Ws[i], 0, 1, c, 0, 0, 0, 0, 0),
                                                           C.add_rmsnorm(normed, resid, out, nw, 1e-5)))
                        else:
                            out = torch.empty(s, M, N, device=dev)
                            fn = (lambda i, out=out, c=c, s=s: (C.skinny_gemm(out, x, Ws[i], 1, s, c, 0, 0, 0, 0, 0),
                                                                C.splitk_add_rmsnorm(normed, resid, out, s, nw, 1e-5)))
                    else:
                        if s == 1:
                            out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
                            fn = (lambda i, out=out, c=c: (C.skinny_gemm(out, x, Ws[i], 0, 1, c, 0, 0, 0, 0, 0),
                                                           rope(out)))
                        else:
                            out = torch.empty(s, M, N, device=dev)
                            qb = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
                            fn = (lambda i, out=out, c=c, s=s, qb=qb: (
                                C.skinny_gemm(out, x, Ws[i], 1, s, c, 0, 0, 0, 0, 0), rope(qb, out)))
                    t = timeit(fn, n_rot, a.iters)
                    if a.all:
                        print(json.dumps({"shape": name, "M": M, "cfg": c, "split": s, "us": round(t, 2)}), flush=True)
                    if best is None or t < best[0]:
                        best = (t, c, s, blocks)
            row = {"shape": name, "N": N, "K": K, "M": M, "lib_us": round(lib, 2)}
            if best is not None:
                row.update(best_us=round(best[0], 2), cfg=best[1], split=best[2], blocks=best[3],
                           speedup=round(lib / best[0], 3))
            win = best is not None and best[0] < 0.97 * lib
            entry["by_m"][str(M)] = [best[1], best[2]] if win else "lib"
            print(json.dumps(row), flush=True)
        del Ws
        torch.cuda.empty_cache()
    out = a.out or os.path.join(os.path.dirname(ops.__file__), "..", "assets", "skinny_gemm_gfx950.json")
    if a.merge:
        with open(a.merge) as f:
            old = json.load(f)["table"]
        old.update(table)
        table = old
    with open(out, "w") as f:
        json.dump({"arch": "gfx950", "model": a.model if not a.merge else "llama3-8b; llama3-70b TP=8 ranks", "note": "decode-shape GEMM choice per (N x K, M): "
                   "[cfg, split] of csrc/kernels/gemm_skinny.hip or 'lib'; benchmarks/skinny_table.py",
                   "table": table}, f, indent=1)
    print("table written:", os.path.abspath(out), flush=True)


if __name__ == "__main__":
    main()
