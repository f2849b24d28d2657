#!/usr/bin/env python3
"""Micro-benchmark of one steady-state mixed step of the RAG bench on Llama-3-8B:
``--decode`` running sequences at ``--ctx`` tokens each (one decode row apiece) plus a
``--prefill``-token chunk of a new prompt, through the full 32-layer forward.

Compares the single-stream mixed forward (decode rows ride on the prefill GEMMs) with
``LlamaModel.forward_split`` (decode rows and prefill rows as independent groups on two
HIP streams), checks that both give the same hidden rows, and reports ms per step.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from nv_genai_amd import ops  # noqa: E402
from nv_genai_amd.models.config import llama_config  # noqa: E402
from nv_genai_amd.models.llama import AttnMeta, LlamaModel  # noqa: E402
from nv_genai_amd.ops.gemm_tuning import use_tuned_gemms  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--decode", type=int, default=256)
    ap.add_argument("--ctx", type=int, default=1330)
    ap.add_argument("--prefill", default="1170", help="comma list of prefill chunk lengths")
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    use_tuned_gemms()
    dev = torch.device("cuda")
    cfg = llama_config(args.model)
    m = LlamaModel(cfg, dev, seed=0)
    B, L = args.decode, args.ctx
    pre = [int(x) for x in args.prefill.split(",")]
    pages_d = (L + 63) // 64
    nblk = B * pages_d + sum((p + 63) // 64 for p in pre) + 8
    m.allocate_kv_cache(nblk)
    m.k_cache.normal_(0, 1)
    m.v_cache.normal_(0, 1)
    n = B + len(pre)
    mb = 8192 // 64   # engine layout: block tables as wide as max_model_len
    bt = torch.zeros(n, mb, dtype=torch.int32)
    o = 0
    for i in range(B):
        bt[i, :pages_d] = torch.arange(o, o + pages_d)
        o += pages_d
    for j, p in enumerate(pre):
        k = (p + 63) // 64
        bt[B + j, :k] = torch.arange(o, o + k)
        o += k
    ctx = torch.tensor([L] * B + pre, dtype=torch.int32)
    pos = torch.cat([torch.full((B,), L - 1, dtype=torch.int32)] + [torch.arange(p, dtype=torch.int32) for p in pre])
    rows_seq = list(range(B)) + [B + j for j, p in enumerate(pre) for _ in range(p)]
    slots = torch.tensor([int(bt[s, int(pp) // 64]) * 64 + int(pp) % 64 for s, pp in zip(rows_seq, pos.tolist())],
                         dtype=torch.int32)
    cu = torch.tensor([0] + list(torch.tensor([1] * B + pre).cumsum(0).tolist()), dtype=torch.int32)
    T = int(cu[-1])
    ids = torch.randint(0, 30000, (T,), dtype=torch.int32)
    ws = ops.DecodeWorkspace(512, m.hq, m.hkv, 8192, dev)
    meta = AttnMeta(kind="mixed", slots=slots.to(dev), cu_q=cu.to(dev), ctx_lens=ctx.to(dev),
                    block_tables=bt.to(dev), max_q_len=max(pre), max_ctx=8192, decode_ws=ws,
                    n_decode=B, cu_q_prefill=(cu[B:] - B).to(dev))
    ids, pos = ids.to(dev), pos.to(dev)
    sample_idx = (cu[1:] - 1).long().to(dev)

    modes = {"fused": (False, False), "fused_concurrent_attn": (False, True), "split": (True, False)}

    def run(mode):
        m.split_mixed, m.concurrent_attention = modes[mode]
        return m.forward(ids, pos, meta, sample_idx)

    out = {}
    ref = run("fused").float()
    for mode in ("fused_concurrent_attn", "split"):
        got = run(mode).float()
        torch.cuda.synchronize()
        out[f"max_abs_diff_{mode}"] = float((ref - got).abs().max())
    out["ref_abs_max"] = float(ref.abs().max())
    for mode in list(modes) * 2:
        for _ in range(2):
            run(mode)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(args.iters):
            run(mode)
        b.record()
        torch.cuda.synchronize()
        out[f"{mode}_ms"] = round(a.elapsed_time(b) / args.iters, 3)
    out.update(decode=B, ctx=L, prefill=pre, tokens=T)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
