"""Two-batch overlap probe for the decode step (llama3-8b shapes, GQA 32 / 8, head_dim 128).

A decode layer at 256 rows is two kinds of work in sequence: the paged attention, bound by the
HBM stream of the KV pages, and the projection GEMMs, bound by the L2 -> CU intake of weight
and activation tiles (docs/performance.md). Split the batch into two halves and the attention
of one half could run beside the GEMMs of the other on a second stream (each layer: [attn(A) |
GEMMs(B)] then [attn(B) | GEMMs(A)]), if the two bottlenecks are separate enough to overlap.
The price: every weight byte is streamed twice per layer (two half-batch GEMMs).

This measures, with weights rotating past the MALL:
  full   = attn(2h) + GEMMs(2h)            (today's layer, one stream)
  halves = attn(h), GEMMs(h) alone
  pair   = attn(h) on stream 1 | GEMMs(h) on stream 2, both launched, then joined
and prints the per-layer time of the two-batch schedule (2 x pair) against full.
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

HQ, HKV, D, H, F = 32, 8, 128, 4096, 14336


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=256, help="full batch (two halves of rows / 2)")
    ap.add_argument("--ctx", type=int, default=1400)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    use_tuned_gemms()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    R, h = a.rows, a.rows // 2
    pages = -(-a.ctx // 64)
    nblk = R * pages
    kc = torch.randn(nblk, HKV, 64, D, device=dev, dtype=torch.bfloat16, generator=g)
    vc = torch.randn(nblk, HKV, D, 64, device=dev, dtype=torch.bfloat16, generator=g)
    bt = torch.randperm(nblk, device=dev, generator=g).to(torch.int32).view(R, pages)
    ctx = torch.full((R,), a.ctx, device=dev, dtype=torch.int32)
    q = torch.randn(R, HQ * D, device=dev, dtype=torch.bfloat16, generator=g)
    scale = D ** -0.5
    ws = {n: ops.DecodeWorkspace(n, HQ, HKV, a.ctx, dev) for n in (R, h)}

    # one layer's projections, rotated over enough copies to miss the 256 MB MALL
    shapes = {"wqkv": (6144, H), "wo": (H, H), "wgu": (2 * F, H), "wd": (H, F)}
    per_layer = sum(n * k * 2 for n, k in shapes.values())
    nrot = max(2, math.ceil(640e6 / per_layer))
    W = [{k: torch.randn(n, kk, device=dev, dtype=torch.bfloat16, generator=g) * 0.02
          for k, (n, kk) in shapes.items()} for _ in range(nrot)]
    nw = torch.ones(H, device=dev, dtype=torch.bfloat16)
    tab = ops.skinny.table()
    xs = {n: torch.randn(n, H, device=dev, dtype=torch.bfloat16, generator=g) for n in (R, h)}
    res = {n: torch.randn(n, H, device=dev, dtype=torch.bfloat16, generator=g) for n in (R, h)}
    att = {n: torch.randn(n, HQ * D, device=dev, dtype=torch.bfloat16, generator=g) for n in (R, h)}

    def lin(x, w, name, M):
        N, K = shapes[name]
        pk = tab.pick(N, K, M)
        if name == "wgu":
            if pk is None:
                return ops.silu_mul(x @ w.t())
            return (ops.skinny_gemm(x, w, pk[0], 1, 2) if pk[1] == 1
                    else ops.splitk_swiglu(ops.skinny_gemm(x, w, pk[0], pk[1], 1)))
        if pk is None:
            return x @ w.t()
        if pk[1] == 1:
            return ops.skinny_gemm(x, w, pk[0], 1, 0)
        return ops.skinny_gemm(x, w, pk[0], pk[1], 1)

    def gemms(n, i, rows=None):
        """The layer's projections for n rows (o + add/RMSNorm, gate/up + SwiGLU, down +
        add/RMSNorm, next layer's q/k/v)."""
        w = W[i % nrot]
        x, r = xs[n], res[n]
        o = lin(att[n], w["wo"], "wo", n)
        hn = ops.splitk_add_rmsnorm(r, o, nw, 1e-5) if o.dim() == 3 else ops.add_rmsnorm(r, o, nw, 1e-5)
        hh = lin(hn, w["wgu"], "wgu", n)
        d = lin(hh, w["wd"], "wd", n)
        xn = ops.splitk_add_rmsnorm(r, d, nw, 1e-5) if d.dim() == 3 else ops.add_rmsnorm(r, d, nw, 1e-5)
        qkv = lin(xn, w["wqkv"], "wqkv", n)
        return qkv

    def attn(n, off=0):
        return ops.decode_attention(q[off:off + n], kc, vc, bt[off:off + n], ctx[off:off + n], HQ, HKV,
                                    a.ctx, scale, ws=ws[n])

    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    main_s = torch.cuda.current_stream(dev)

    def pair(i):
        s1.wait_stream(main_s)
        s2.wait_stream(main_s)
        with torch.cuda.stream(s1):
            attn(h, 0)
        with torch.cuda.stream(s2):
            gemms(h, i)
        main_s.wait_stream(s1)
        main_s.wait_stream(s2)

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

    out = {"rows": R, "ctx": a.ctx, "rotations": nrot}
    for rnd in range(2):   # interleaved rounds: the spread shows the noise
        r = {"attn_full_us": timeit(lambda i: attn(R)), "gemms_full_us": timeit(lambda i: gemms(R, i)),
             "attn_half_us": timeit(lambda i: attn(h)), "gemms_half_us": timeit(lambda i: gemms(h, i)),
             "pair_us": timeit(pair)}
        r["layer_today_us"] = r["attn_full_us"] + r["gemms_full_us"]
        r["layer_two_batch_us"] = 2 * r["pair_us"]
        r["gain"] = 1 - r["layer_two_batch_us"] / r["layer_today_us"]
        out[f"round{rnd}"] = {k: round(v, 2) if isinstance(v, float) else v for k, v in r.items()}
        print(json.dumps({**{k: v for k, v in out.items() if not k.startswith("round")},
                          "round": rnd, **out[f"round{rnd}"]}), flush=True)


if __name__ == "__main__":
    main()
