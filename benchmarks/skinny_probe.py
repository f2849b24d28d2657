"""Time chosen (cfg, split) pairs of the decode-shape GEMM on one projection WITH its model
consumer (SwiGLU / split-K SwiGLU for gate/up, split-K add + RMSNorm for o / down, the
RoPE-less slab sum for q/k/v), weights rotating past the MALL:
``--shape gate_up --m 256 --pairs 13:1,17:2,18:2``. One JSON line per pair."""
import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from nv_genai_amd import ops  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "lm_head": (128256, 4096)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="gate_up")
    ap.add_argument("--m", type=int, default=256)
    ap.add_argument("--pairs", required=True)
    ap.add_argument("--iters", type=int, default=40)
    a = ap.parse_args()
    N, K = SHAPES[a.shape]
    dev = torch.device("cuda")
    n_rot = max(2, math.ceil(640e6 / (N * K * 2)))
    Ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(n_rot)]
    x = torch.randn(a.m, K, device=dev, dtype=torch.bfloat16)
    resid = torch.randn(a.m, N, device=dev, dtype=torch.bfloat16)
    nw = torch.ones(N, device=dev, dtype=torch.bfloat16)

    def run(i, cfg, split):
        w = Ws[i % n_rot]
        if a.shape == "gate_up":
            if split == 1:
                return ops.skinny_gemm(x, w, cfg, 1, 2)
            return ops.splitk_swiglu(ops.skinny_gemm(x, w, cfg, split, 1))
        if a.shape in ("o", "down"):
            return ops.splitk_add_rmsnorm(resid, ops.skinny_gemm(x, w, cfg, split, 1), nw, 1e-5)
        return ops.skinny_gemm(x, w, cfg, split, 1 if split > 1 or a.shape == "lm_head" else 0)

    def lib(i):
        w = Ws[i % n_rot]
        y = x @ w.t()
        if a.shape == "gate_up":
            return ops.silu_mul(y)
        if a.shape in ("o", "down"):
            return ops.add_rmsnorm(resid, y, nw, 1e-5)
        return y

    def timeit(fn):
        for i in range(3):
            fn(i)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(a.iters):
            fn(i)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.iters * 1e3

    print(json.dumps({"shape": a.shape, "M": a.m, "lib_us": round(timeit(lib), 2)}), flush=True)
    for p in a.pairs.split(","):
        cfg, split = (int(v) for v in p.split(":"))
        us = timeit(lambda i: run(i, cfg, split))
        print(json.dumps({"shape": a.shape, "M": a.m, "cfg": cfg, "split": split, "us": round(us, 2),
                          "tile": ops.kernels().skinny_cfg(cfg)}), flush=True)


if __name__ == "__main__":
    main()
