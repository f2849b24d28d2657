"""Intra-GPU overlap probe: can the decode rows' HBM-bound work (paged decode attention over
~1.4K-token contexts, weight-streaming M=256 GEMMs) run beside the prefill rows' MFMA-bound
GEMMs on the same MI355X, and what does a mixed step gain from it?

A headline mixed step (bench.py) carries ~250 decode rows and ~1.2K prefill tokens. The
engine runs them as ONE forward (M ≈ 1.4K GEMMs, decode and prefill attention side by side).
The alternative measured here splits the step into two independent forwards — decode rows
and prefill rows touch disjoint sequences, so nothing couples them but the shared weights —
on two HIP streams, so the hardware interleaves memory-bound and compute-bound kernels.

Emulated layer (Llama-3-8B shapes, 32 distinct layers of weights so every GEMM streams its
weights from HBM): add+RMSNorm, QKV GEMM, attention, O GEMM, add+RMSNorm, gate/up GEMM,
SiLU·mul, down GEMM. RoPE / KV append / sampling are left out (~2 % of the step).

Variants (GPU time per 32-layer step, CUDA events):
  fused      one forward over Md + Mp rows (the engine today): decode attention on the main
             stream, prefill attention on a side stream
  split_ser  the two forwards back to back on one stream
  split_conc the two forwards on two streams
  split_graph split_conc captured in one hipGraph (fork / join)
  *_prio     the decode stream at high priority
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from nv_genai_amd import ops  # noqa: E402
from nv_genai_amd.ops.gemm_tuning import use_tuned_gemms  # noqa: E402


def paged(lens, Hkv, D, dev, width=None):
    nb = sum((l + 63) // 64 for l in lens)
    kc = torch.randn(nb, Hkv, 64, D, device=dev, dtype=torch.bfloat16)
    vc = torch.randn(nb, Hkv, D, 64, device=dev, dtype=torch.bfloat16)
    mb = width or max((l + 63) // 64 for l in lens)
    bt = torch.zeros(len(lens), mb, dtype=torch.int32, device=dev)
    o = 0
    for i, l in enumerate(lens):
        n = (l + 63) // 64
        bt[i, :n] = torch.arange(o, o + n, dtype=torch.int32)
        o += n
    return kc, vc, bt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--decode-rows", type=int, default=256)
    ap.add_argument("--decode-ctx", type=int, default=1400)
    ap.add_argument("--prefill", default="1168", help="comma-separated prompt lengths of the step")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--no-tuned", action="store_true")
    ap.add_argument("--micro", action="store_true",
                    help="decode-only step: the decode rows as ONE forward vs two half-batch forwards "
                         "on two streams (HBM-bound attention of one half beside the latency-bound "
                         "small-M GEMMs of the other)")
    args = ap.parse_args()
    if args.micro:
        return micro(args)
    dev = "cuda"
    tuned = False if args.no_tuned else use_tuned_gemms()
    H, I, Hq, Hkv, D, eps = 4096, 14336, 32, 8, 128, 1e-5
    QKV = (Hq + 2 * Hkv) * D
    L = args.layers
    Md = args.decode_rows
    plens = [int(x) for x in args.prefill.split(",") if x]
    Mp = sum(plens)
    g = torch.Generator(device=dev).manual_seed(0)

    def w(n, k):
        return (torch.randn(n, k, device=dev, dtype=torch.bfloat16, generator=g) * k ** -0.5)

    Ws = [dict(qkv=w(QKV, H), o=w(H, Hq * D), gu=w(2 * I, H), d=w(H, I),
               n1=torch.ones(H, device=dev, dtype=torch.bfloat16),
               n2=torch.ones(H, device=dev, dtype=torch.bfloat16)) for _ in range(L)]
    # decode KV: one cache shared by the layers (1.5 GB per layer pass >> the 256 MB MALL, so
    # every layer still streams it from HBM)
    kcd, vcd, btd = paged([args.decode_ctx] * Md, Hkv, D, dev, width=8192 // 64)
    ctxd = torch.full((Md,), args.decode_ctx, dtype=torch.int32, device=dev)
    wsd = ops.DecodeWorkspace(Md, Hq, Hkv, 8192, torch.device(dev))
    kcp, vcp, btp = paged(plens, Hkv, D, dev)
    cup = torch.tensor([0] + torch.tensor(plens).cumsum(0).tolist(), dtype=torch.int32, device=dev)
    ctxp = torch.tensor(plens, dtype=torch.int32, device=dev)
    scale = D ** -0.5

    def bufs(M):
        return dict(x=torch.randn(M, H, device=dev, dtype=torch.bfloat16, generator=g) * 0.1,
                    r=torch.zeros(M, H, device=dev, dtype=torch.bfloat16),
                    a=torch.empty(M, Hq * D, device=dev, dtype=torch.bfloat16),
                    h=torch.empty(M, I, device=dev, dtype=torch.bfloat16))

    bd, bp, bf = bufs(Md), bufs(Mp), bufs(Md + Mp)

    def layer_stack(b, attn):
        x, r = b["x"], b["r"]
        for W in Ws:
            hn = ops.add_rmsnorm(r, x, W["n1"], eps)
            qkv = F.linear(hn, W["qkv"])
            attn(qkv, b["a"])
            o = F.linear(b["a"], W["o"])
            hn = ops.add_rmsnorm(r, o, W["n2"], eps)
            gu = F.linear(hn, W["gu"])
            ops.silu_mul(gu, out=b["h"])
            x = F.linear(b["h"], W["d"])
        return x

    def attn_decode(qkv, out):
        ops.decode_attention(qkv[:, : Hq * D], kcd, vcd, btd, ctxd, Hq, Hkv, 8192, scale,
                             out=out, ws=wsd)

    def attn_prefill(qkv, out):
        ops.prefill_attention_paged(qkv[:, : Hq * D], kcp, vcp, btp, cup, ctxp, Hq, Hkv, D,
                                    max(plens), scale, out=out)

    side = torch.cuda.Stream()

    def attn_fused(qkv, out):
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            attn_prefill(qkv[Md:], out[Md:])
        attn_decode(qkv[:Md], out[:Md])
        cur.wait_stream(side)

    s_dec = torch.cuda.Stream()
    s_pre = torch.cuda.Stream()
    s_dec_hi = torch.cuda.Stream(priority=-1)

    def fused():
        layer_stack(bf, attn_fused)

    def split_ser():
        layer_stack(bd, attn_decode)
        layer_stack(bp, attn_prefill)

    def split_conc(sd=s_dec):
        cur = torch.cuda.current_stream()
        sd.wait_stream(cur)
        s_pre.wait_stream(cur)
        with torch.cuda.stream(sd):
            layer_stack(bd, attn_decode)
        with torch.cuda.stream(s_pre):
            layer_stack(bp, attn_prefill)
        cur.wait_stream(sd)
        cur.wait_stream(s_pre)

    def decode_only():
        layer_stack(bd, attn_decode)

    def prefill_only():
        layer_stack(bp, attn_prefill)

    def timeit(fn, iters):
        fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / iters

    res = {"config": {"layers": L, "decode_rows": Md, "decode_ctx": args.decode_ctx,
                      "prefill": plens, "tuned_gemms": tuned}}
    variants = [("decode_only", decode_only), ("prefill_only", prefill_only), ("fused", fused),
                ("split_ser", split_ser), ("split_conc", split_conc),
                ("split_conc_prio", lambda: split_conc(s_dec_hi))]
    for name, fn in variants:
        res[name + "_ms"] = round(timeit(fn, args.iters), 3)
        print(json.dumps({name: res[name + "_ms"]}), flush=True)
    for name, fn in (("fused_graph", fused), ("split_graph", split_conc),
                     ("split_graph_prio", lambda: split_conc(s_dec_hi))):
        gr = torch.cuda.CUDAGraph()
        fn()
        torch.cuda.synchronize()
        with torch.cuda.graph(gr):
            fn()
        res[name + "_ms"] = round(timeit(gr.replay, args.iters), 3)
        print(json.dumps({name: res[name + "_ms"]}), flush=True)
        del gr
    res["gain_conc_vs_fused"] = round(res["fused_ms"] / res["split_conc_ms"], 3)
    res["gain_graph_vs_fused_graph"] = round(res["fused_graph_ms"] / res["split_graph_ms"], 3)
    print(json.dumps(res))


def micro(args):
    dev = "cuda"
    tuned = False if args.no_tuned else use_tuned_gemms()
    H, I, Hq, Hkv, D, eps = 4096, 14336, 32, 8, 128, 1e-5
    QKV = (Hq + 2 * Hkv) * D
    Md, hm = args.decode_rows, args.decode_rows // 2
    g = torch.Generator(device=dev).manual_seed(0)

    def w(n, k):
        return (torch.randn(n, k, device=dev, dtype=torch.bfloat16, generator=g) * k ** -0.5)

    Ws = [dict(qkv=w(QKV, H), o=w(H, Hq * D), gu=w(2 * I, H), d=w(H, I),
               n1=torch.ones(H, device=dev, dtype=torch.bfloat16),
               n2=torch.ones(H, device=dev, dtype=torch.bfloat16)) for _ in range(args.layers)]
    kcd, vcd, btd = paged([args.decode_ctx] * Md, Hkv, D, dev, width=8192 // 64)
    ctxd = torch.full((Md,), args.decode_ctx, dtype=torch.int32, device=dev)
    scale = D ** -0.5
    parts = {"all": (0, Md), "a": (0, hm), "b": (hm, Md)}
    wss = {k: ops.DecodeWorkspace(hi - lo, Hq, Hkv, 8192, torch.device(dev)) for k, (lo, hi) in parts.items()}

    def bufs(M):
        return dict(x=torch.randn(M, H, device=dev, dtype=torch.bfloat16, generator=g) * 0.1,
                    r=torch.zeros(M, H, device=dev, dtype=torch.bfloat16),
                    a=torch.empty(M, Hq * D, device=dev, dtype=torch.bfloat16),
                    h=torch.empty(M, I, device=dev, dtype=torch.bfloat16))

    B = {k: bufs(hi - lo) for k, (lo, hi) in parts.items()}

    def stack(k):
        lo, hi = parts[k]
        b = B[k]
        x, r = b["x"], b["r"]
        for W in Ws:
            hn = ops.add_rmsnorm(r, x, W["n1"], eps)
            qkv = F.linear(hn, W["qkv"])
            ops.decode_attention(qkv[:, : Hq * D], kcd, vcd, btd[lo:hi], ctxd[lo:hi], Hq, Hkv, 8192, scale,
                                 out=b["a"], ws=wss[k])
            o = F.linear(b["a"], W["o"])
            hn = ops.add_rmsnorm(r, o, W["n2"], eps)
            gu = F.linear(hn, W["gu"])
            ops.silu_mul(gu, out=b["h"])
            x = F.linear(b["h"], W["d"])
        return x

    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()

    def one():
        stack("all")

    def halves_ser():
        stack("a")
        stack("b")

    def halves_conc():
        cur = torch.cuda.current_stream()
        sa.wait_stream(cur)
        sb.wait_stream(cur)
        with torch.cuda.stream(sa):
            stack("a")
        with torch.cuda.stream(sb):
            stack("b")
        cur.wait_stream(sa)
        cur.wait_stream(sb)

    def timeit(fn, iters):
        fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / iters

    res = {"config": {"layers": args.layers, "decode_rows": Md, "decode_ctx": args.decode_ctx, "tuned_gemms": tuned}}
    for name, fn in (("one_forward", one), ("halves_serial", halves_ser), ("halves_two_streams", halves_conc)):
        gr = torch.cuda.CUDAGraph()
        fn()
        torch.cuda.synchronize()
        with torch.cuda.graph(gr):
            fn()
        res[name + "_graph_ms"] = round(timeit(gr.replay, args.iters), 3)
        print(json.dumps({name: res[name + "_graph_ms"]}), flush=True)
        del gr
    res["gain_two_streams"] = round(res["one_forward_graph_ms"] / res["halves_two_streams_graph_ms"], 3)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
