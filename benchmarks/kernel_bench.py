"""Micro-benchmarks of the hand-written hot kernels at serving shapes (Llama-3-8B):
prefill attention (paged, causal, GQA 32/8, D=128), decode attention, sampling, and the
1M x 1024 flat-index search (MFMA scoring + radix top-k)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from nv_genai_amd import ops  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3  # us


def timeit_graph(fn, iters=20):
    """Per-call time of ``iters`` calls captured in one hipGraph and replayed: the form the
    engine runs decode in (no per-launch host overhead between the kernels)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(3):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / (3 * iters) * 1e3  # us


def paged_setup(lens, Hkv=8, D=128, dev="cuda", width=None):
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
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="", help="rope | norm | bw | prefill | decode | decode_small | sample | search (default: all)")
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    global timeit
    _t = timeit
    timeit = lambda fn: _t(fn, args.iters)  # noqa: E731
    dev = "cuda"
    Hq, Hkv, D = 32, 8, 128
    out = {}
    if args.only in ("", "rope"):
        cs = ops.rope_cos_sin(8192, D).to(dev)
        nb = 4096
        kc = torch.zeros(nb, Hkv, 64, D, device=dev, dtype=torch.bfloat16)
        vc = torch.zeros(nb, Hkv, D, 64, device=dev, dtype=torch.bfloat16)
        for T, kind in ((1536, "prefill"), (256, "decode"), (1190, "mixed")):
            qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device=dev).to(torch.bfloat16)
            pos = torch.arange(T, dtype=torch.int32, device=dev) % 4096
            scattered = torch.randperm(nb, device=dev)[:T] * 64 + 17
            if kind == "prefill":
                slots = torch.arange(T, device=dev)
            elif kind == "decode":
                slots = scattered
            else:   # a mixed step: 256 decode rows, then one prompt's contiguous slots
                slots = torch.cat([scattered[:256], torch.arange(T - 256, device=dev) + 64 * 4000])
            slots = slots.to(torch.int32)
            us = timeit(lambda: ops.rope_cache_(qkv, pos, cs, slots, kc, vc, Hq, Hkv, D))
            moved = T * (Hq + 2 * Hkv) * D * 2 + T * (Hq + Hkv) * D * 2 + 2 * T * Hkv * D * 2
            out[f"rope_cache_T{T}_{kind}"] = {"us": round(us, 1), "TBps": round(moved / us / 1e6, 2)}
        del kc, vc
        if args.only == "rope":
            print(json.dumps(out))
            return
    if args.only in ("", "norm"):
        # residual add + RMSNorm at decode / mixed / full-budget step sizes (Llama-3-8B width):
        # add + RMSNorm at the headline's step sizes
        w = torch.randn(4096, device=dev).to(torch.bfloat16)
        for T in (256, 1426, 4352):
            r = torch.randn(T, 4096, device=dev).to(torch.bfloat16)
            dlt = torch.randn(T, 4096, device=dev).to(torch.bfloat16)
            o = torch.empty_like(r)
            us = timeit(lambda: ops.add_rmsnorm(r, dlt, w, 1e-5, out=o))
            out[f"add_rmsnorm_{T}x4096"] = {"us": round(us, 1), "TBps": round(4 * T * 4096 * 2 / us / 1e6, 2)}
        if args.only == "norm":
            print(json.dumps(out))
            return
    if args.only in ("", "bw"):
        # HBM read ceiling of this box for the bandwidth-bound kernels: a 2 GiB bf16 slab
        # reduced by PyTorch (read-only stream) and copied device to device (read + write)
        X = torch.empty(1 << 30, dtype=torch.bfloat16, device=dev).normal_()
        Y = torch.empty_like(X)
        us_sum = timeit(lambda: X.sum(dtype=torch.float32))
        us_cp = timeit(lambda: Y.copy_(X))
        out["hbm_read_sum_2GiB"] = {"us": round(us_sum, 1), "TBps": round(X.numel() * 2 / us_sum / 1e6, 2)}
        out["hbm_copy_2GiB"] = {"us": round(us_cp, 1), "TBps_read_plus_write": round(2 * X.numel() * 2 / us_cp / 1e6, 2)}
        del X, Y
        if args.only == "bw":
            print(json.dumps(out))
            return
    if args.only in ("", "search"):
        N, Dx = 1_000_000, 1024
        X = torch.nn.functional.normalize(torch.randn(N, Dx, device=dev), dim=1).to(torch.bfloat16)
        bias = torch.zeros(N, device=dev)
        for nq in (1, 8, 64):
            Q = torch.nn.functional.normalize(torch.randn(nq, Dx, device=dev), dim=1).to(torch.bfloat16)
            us = timeit(lambda: ops.score(Q, X, None, 1.0))
            us_all = timeit(lambda: ops.topk(ops.score(Q, X, None, 1.0), 4))
            us_f = timeit(lambda: ops.search_topk(Q, X, bias, 1.0, 4))
            ops.kernels().set_kernel_form("search_dma", 0)    # the register-load form
            us_reg = timeit(lambda: ops.search_topk(Q, X, bias, 1.0, 4))
            ops.kernels().set_kernel_form("search_dma", 1)
            out[f"search_1Mx1024_q{nq}"] = {"reg_us": round(us_reg, 1),
                                             "reg_TBps": round(N * Dx * 2 / us_reg / 1e6, 2),
                                             "score_us": round(us, 1), "score_TBps": round(N * Dx * 2 / us / 1e6, 2),
                                             "score_topk_us": round(us_all, 1),
                                             "fused_us": round(us_f, 1),
                                             "fused_TBps": round(N * Dx * 2 / us_f / 1e6, 2),
                                             "fused_vs_score_only": round(us_f / us, 3)}
        # one 1.25M-vector shard of the 10M index over 8 GPUs
        Xs = X[:1_000_000]
        Xs = torch.cat([Xs, Xs[:250_000]])
        bs = torch.zeros(Xs.shape[0], device=dev)
        for nq in (8, 64):
            Q = torch.nn.functional.normalize(torch.randn(nq, Dx, device=dev), dim=1).to(torch.bfloat16)
            us_f = timeit(lambda: ops.search_topk(Q, Xs, bs, 1.0, 4))
            ops.kernels().set_kernel_form("search_dma", 0)
            us_reg = timeit(lambda: ops.search_topk(Q, Xs, bs, 1.0, 4))
            ops.kernels().set_kernel_form("search_dma", 1)
            out[f"search_shard1.25Mx1024_q{nq}"] = {"reg_us": round(us_reg, 1), "fused_us": round(us_f, 1),
                                                    "fused_TBps": round(Xs.numel() * 2 / us_f / 1e6, 2)}
        del Xs, bs
        # IVF-Flat, the reference's GPU_IVF_FLAT nlist 64 / nprobe 16 over 1M vectors
        from nv_genai_amd.index.ivf import IVFFlatIndex

        ivf = IVFFlatIndex(Dx, nlist=64, nprobe=16, metric="cosine", device=dev)
        ivf.train(X[:200_000].float(), iters=5)
        ivf.add(X, torch.arange(N))
        for nq in (1, 8, 64):
            Q = torch.nn.functional.normalize(torch.randn(nq, Dx, device=dev), dim=1)
            us_i = timeit(lambda: ivf.search(Q, 4))
            ops.kernels().set_kernel_form("search_dma", 0)
            us_ir = timeit(lambda: ivf.search(Q, 4))
            ops.kernels().set_kernel_form("search_dma", 1)
            out[f"ivf_1Mx1024_nlist64_nprobe16_q{nq}"] = {"us": round(us_i, 1), "reg_us": round(us_ir, 1)}
        del ivf
        del X
        if args.only == "search":
            print(json.dumps(out))
            return
    for name, lens, qls in (("prefill_1x1196", [1196], None), ("prefill_2x1200", [1200] * 2, None),
                            ("prefill_3x1200", [1200] * 3, None), ("prefill_6x1200", [1200] * 6, None),
                            ("prefill_27x1200", [1200] * 27, None), ("prefill_4x4096", [4096] * 4, None),
                            ("prefill_chunk_940_of_1200", [1200], [940]),
                            ("prefill_chunk_1024_of_8192", [8192], [1024])):
        if args.only and args.only != "prefill":
            break
        qls = qls or lens
        kc, vc, bt = paged_setup(lens)
        T = sum(qls)
        q = torch.randn(T, Hq * D, device=dev, dtype=torch.bfloat16)
        cu = torch.tensor([0] + list(torch.tensor(qls).cumsum(0).tolist()), dtype=torch.int32, device=dev)
        ctx = torch.tensor(lens, dtype=torch.int32, device=dev)
        # causal FLOPs: query i of a ql-row chunk ending at ctx sees ctx - ql + i + 1 keys
        flops = sum(2 * 2 * (ql * (c - ql) + ql * (ql + 1) / 2) * D * Hq for c, ql in zip(lens, qls))
        out[name] = {}
        for impl, tag in ((0, "auto"), (4, "auto_alone"), (1, "mfma16"), (2, "mfma32"), (3, "mfma32_ks2"),
                          (5, "mfma32_w8"), (6, "mfma32_stg")):
            us = timeit(lambda: ops.prefill_attention_paged(q, kc, vc, bt, cu, ctx, Hq, Hkv, D, max(qls),
                                                            D ** -0.5, impl=impl))
            out[name][tag] = {"us": round(us, 1), "TFLOPs": round(flops / us / 1e6, 1)}
    B, L = 256, 1400
    if args.only == "prefill":
        print(json.dumps(out))
        return
    if args.only in ("", "decode"):
        kc, vc, bt = paged_setup([L] * B, width=8192 // 64)
        q = torch.randn(B, Hq * D, device=dev, dtype=torch.bfloat16)
        ctx = torch.full((B,), L, dtype=torch.int32, device=dev)
        for ppp in (None, 16, 32):
            ws = ops.DecodeWorkspace(B, Hq, Hkv, 8192, torch.device(dev), ppp)
            us = timeit(lambda: ops.decode_attention(q, kc, vc, bt, ctx, Hq, Hkv, 8192, D ** -0.5, ws=ws))
            out[f"decode_256x1400_ppp{ppp}"] = {"us": round(us, 1), "TBps": round(B * L * Hkv * D * 2 * 2 / us / 1e6, 2)}
        # DMA kernel forms (NGA_DECODE_DMA 1: whole page per wave slot, 2: half-page ring),
        # interleaved 3 times at the headline's and smaller batch sizes
        for Bs in (256, 64, 16):
            kcx, vcx, btx = (kc, vc, bt) if Bs == B else paged_setup([L] * Bs, width=8192 // 64)
            qx = q[:Bs].contiguous()
            ctxx = torch.full((Bs,), L, dtype=torch.int32, device=dev)
            wsx = ops.DecodeWorkspace(Bs, Hq, Hkv, 8192, torch.device(dev))
            res = {"1": [], "2": []}
            for _ in range(3):
                for form in ("1", "2"):
                    ops.kernels().set_kernel_form("decode_dma", int(form))
                    res[form].append(round(timeit_graph(lambda: ops.decode_attention(
                        qx, kcx, vcx, btx, ctxx, Hq, Hkv, 8192, D ** -0.5, ws=wsx)), 1))
            ops.kernels().set_kernel_form("decode_dma", 1)
            out[f"decode_{Bs}x1400_dma_forms"] = {
                "whole_page_us": res["1"], "ring_us": res["2"],
                "TBps_whole_ring": [round(Bs * L * Hkv * D * 4 / min(res[f]) / 1e6, 2) for f in ("1", "2")]}
        # page placement: the same 256 x 1,400 rows with their pages spread over a serving-size
        # cache (10,752 blocks per layer, as the headline's 30% KV fraction gives) — in order
        # per sequence, and in a random permutation (what an LRU-recycled steady state gives)
        nbig = 10752
        kcb = torch.randn(nbig, Hkv, 64, D, device=dev, dtype=torch.bfloat16)
        vcb = torch.randn(nbig, Hkv, D, 64, device=dev, dtype=torch.bfloat16)
        npg = (L + 63) // 64
        g = torch.Generator().manual_seed(3)
        for tag, order in (("spread", torch.arange(B * npg) * (nbig // (B * npg))),
                           ("random", torch.randperm(nbig, generator=g)[: B * npg])):
            btb = torch.zeros(B, 8192 // 64, dtype=torch.int32, device=dev)
            btb[:, :npg] = order.view(B, npg).to(torch.int32).to(dev)
            ws = ops.DecodeWorkspace(B, Hq, Hkv, 8192, torch.device(dev))
            us = timeit(lambda: ops.decode_attention(q, kcb, vcb, btb, ctx, Hq, Hkv, 8192, D ** -0.5, ws=ws))
            out[f"decode_256x1400_pages_{tag}"] = {"us": round(us, 1), "TBps": round(B * L * Hkv * D * 2 * 2 / us / 1e6, 2)}
        del kcb, vcb
        # fp8 e4m3fn KV pages (half the bytes; TB/s counted on the bytes actually read)
        kc8, vc8 = kc.to(torch.float8_e4m3fn), vc.to(torch.float8_e4m3fn)
        ws = ops.DecodeWorkspace(B, Hq, Hkv, 8192, torch.device(dev))
        us = timeit(lambda: ops.decode_attention(q, kc8, vc8, bt, ctx, Hq, Hkv, 8192, D ** -0.5, ws=ws))
        out["decode_256x1400_fp8kv"] = {"us": round(us, 1), "TBps": round(B * L * Hkv * D * 2 / us / 1e6, 2)}
        del kc8, vc8
        # head_dim 256, MHA (Gemma-7B: 16 q = 16 kv heads)
        kc6, vc6, bt6 = paged_setup([L] * 64, Hkv=16, D=256, width=8192 // 64)
        q6 = torch.randn(64, 16 * 256, device=dev, dtype=torch.bfloat16)
        ctx6 = torch.full((64,), L, dtype=torch.int32, device=dev)
        ws = ops.DecodeWorkspace(64, 16, 16, 8192, torch.device(dev), D=256)
        us = timeit(lambda: ops.decode_attention(q6, kc6, vc6, bt6, ctx6, 16, 16, 8192, 256 ** -0.5, ws=ws))
        out["decode_d256_64x1400"] = {"us": round(us, 1), "TBps": round(64 * L * 16 * 256 * 2 * 2 / us / 1e6, 2)}
        del kc6, vc6
        # adaptive split at other batch sizes (max_ctx 8192 as in the captured decode graphs)
        for Bs in (250, 64, 16, 4):
            kc2, vc2, bt2 = paged_setup([L] * Bs, width=8192 // 64)
            q2 = torch.randn(Bs, Hq * D, device=dev, dtype=torch.bfloat16)
            ctx2 = torch.full((Bs,), L, dtype=torch.int32, device=dev)
            ws = ops.DecodeWorkspace(Bs, Hq, Hkv, 8192, torch.device(dev))
            fn = lambda: ops.decode_attention(q2, kc2, vc2, bt2, ctx2, Hq, Hkv, 8192, D ** -0.5, ws=ws)  # noqa: E731
            us = timeit(fn)
            ug = timeit_graph(fn)
            out[f"decode_{Bs}x1400_auto"] = {"us": round(us, 1), "parts": ws.nparts(Bs),
                                             "TBps": round(Bs * L * Hkv * D * 2 * 2 / us / 1e6, 2),
                                             "graph_us": round(ug, 1),
                                             "graph_TBps": round(Bs * L * Hkv * D * 2 * 2 / ug / 1e6, 2)}
        # Llama-3-70B at TP=8: 8 q heads and 1 KV head per rank (the agent config's decode)
        for Bs in (4, 32):
            kc3, vc3, bt3 = paged_setup([L] * Bs, Hkv=1, width=8192 // 64)
            q3 = torch.randn(Bs, 8 * D, device=dev, dtype=torch.bfloat16)
            ctx3 = torch.full((Bs,), L, dtype=torch.int32, device=dev)
            ws = ops.DecodeWorkspace(Bs, 8, 1, 8192, torch.device(dev))
            fn = lambda: ops.decode_attention(q3, kc3, vc3, bt3, ctx3, 8, 1, 8192, D ** -0.5, ws=ws)  # noqa: E731
            us = timeit(fn)
            ug = timeit_graph(fn)
            out[f"decode_70b_tp8_{Bs}x1400"] = {"us": round(us, 1), "parts": ws.nparts(Bs), "graph_us": round(ug, 1),
                                                "TBps": round(Bs * L * D * 2 * 2 / us / 1e6, 2)}
        if args.only == "decode":
            print(json.dumps(out))
            return
    if args.only == "decode_small":
        # small-batch sweep: register vs LDS-DMA kernel x pages per partition, graph replay
        for name, Bs, Hq_, Hkv_ in (("16x1400", 16, Hq, Hkv), ("4x1400", 4, Hq, Hkv), ("64x1400", 64, Hq, Hkv),
                                    ("70b_tp8_4x1400", 4, 8, 1), ("70b_tp8_32x1400", 32, 8, 1)):
            kc3, vc3, bt3 = paged_setup([L] * Bs, Hkv=Hkv_, width=8192 // 64)
            q3 = torch.randn(Bs, Hq_ * D, device=dev, dtype=torch.bfloat16)
            ctx3 = torch.full((Bs,), L, dtype=torch.int32, device=dev)
            res = {}
            # ppp is in pages of max_ctx 8192 (128 pages): 32 / 43 / 64 / 128 -> 4 / 3 / 2 / 1 partitions
            for ppp in (None, 32, 43, 64, 128):
                ws = ops.DecodeWorkspace(Bs, Hq_, Hkv_, 8192, torch.device(dev), ppp)
                fn = lambda: ops.decode_attention(q3, kc3, vc3, bt3, ctx3, Hq_, Hkv_, 8192, D ** -0.5, ws=ws)  # noqa: E731
                for kern in ("0", "1"):
                    ops.kernels().set_kernel_form("decode_dma", int(kern))
                    res[f"{'dma' if kern == '1' else 'reg'}_ppp{ppp}"] = round(timeit_graph(fn), 1)
                ops.kernels().set_kernel_form("decode_dma", 1)
            best = min(res, key=res.get)
            out[f"decode_small_{name}"] = {"graph_us": res, "best": best,
                                           "best_TBps": round(Bs * L * Hkv_ * D * 4 / res[best] / 1e6, 2)}
        print(json.dumps(out))
        return
    V = 128256
    logits = torch.randn(B, V, device=dev) * 3
    z = lambda v, dt=torch.float32: torch.full((B,), v, dtype=dt, device=dev)  # noqa: E731
    flat = torch.randn(B, V, device=dev) * 0.5
    for nm, (t, k, p) in {"sample_greedy": (0.0, 0, 1.0), "sample_t0.2_p0.7": (0.2, 0, 0.7),
                          "sample_t1_k50": (1.0, 50, 1.0), "sample_t1_k50_p0.9": (1.0, 50, 0.9),
                          "sample_flat_t1_p0.95": (1.0, 0, 0.95),
                          "sample_flat_t1_p0.9999": (1.0, 0, 0.9999)}.items():
        lg = flat if nm.startswith("sample_flat") else logits
        prm = (z(t), z(k, torch.int32), z(p), z(1, torch.int64), z(0, torch.int64))
        us = timeit(lambda: ops.sample(lg, *prm))
        out[nm] = {"us": round(us, 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
