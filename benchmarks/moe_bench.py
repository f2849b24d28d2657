"""MoE MLP micro-benchmark at Mixtral-8x7B layer shapes (H 4096, F 14336, 8 experts, top-2):
the fused HIP path (``ops.moe_ffn``: route + align + gathered grouped MFMA GEMMs with the
SwiGLU epilogue + weighted combine) against the eager PyTorch-ROCm formulation of the same
layer (transformers' MixtralExperts loop: per-expert index_select + hipBLASLt GEMMs +
index_add). Prints one JSON line per token count."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from nv_genai_amd import ops  # noqa: E402


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def eager(x, router, w13, w2, k):
    p = torch.softmax((x @ router.t()).float(), -1)
    w, ids = torch.topk(p, k, -1)
    w = w / w.sum(-1, keepdim=True)
    out = torch.zeros_like(x)
    F = w2.shape[2]
    for e in range(w13.shape[0]):
        tok, slot = torch.where(ids == e)
        if tok.numel() == 0:
            continue
        gu = x[tok] @ w13[e].t()
        h = torch.nn.functional.silu(gu[:, :F]) * gu[:, F:]
        out.index_add_(0, tok, ((h @ w2[e].t()).float() * w[tok, slot, None]).to(x.dtype))
    return out


def main():
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", default="64,256,1536,4096")
    ap.add_argument("--H", type=int, default=4096)
    ap.add_argument("--F", type=int, default=14336)
    ap.add_argument("--E", type=int, default=8)
    ap.add_argument("--k", type=int, default=2)
    ap.add_argument("--gemm-only", action="store_true",
                    help="time the gate|up grouped GEMM alone (NGA_MOE_ABLATE picks a diagnostic build)")
    args = ap.parse_args()
    dev = "cuda"
    H, F, E, k = args.H, args.F, args.E, args.k
    torch.manual_seed(0)
    router = (torch.randn(E, H, device=dev) * 0.02).to(torch.bfloat16)
    w13 = (torch.randn(E, 2 * F, H, device=dev) * 0.02).to(torch.bfloat16)
    w2 = (torch.randn(E, H, F, device=dev) * 0.02).to(torch.bfloat16)
    for T in [int(t) for t in args.tokens.split(",")]:
        x = torch.randn(T, H, device=dev).to(torch.bfloat16)
        ws = ops.MoEWorkspace.get(T, k, E, dev)
        if args.gemm_only:
            C = ops.kernels()
            M = T * k
            bm = 64 if M <= 256 * E else 128
            mt = -(-M // bm) + E
            C.moe_route(x @ router.t(), k, ws.ids, ws.w)
            C.moe_align(ws.ids, ws.w, T, k, 0, E, bm, ws.sorted_tok, ws.sorted_w, ws.inv, ws.tiles, mt)
            h = torch.empty(M, F, dtype=x.dtype, device=dev)
            y = torch.empty(M, H, dtype=x.dtype, device=dev)
            t0 = timeit(lambda: C.moe_gemm(x, w13, ws.sorted_tok, ws.sorted_w, ws.tiles, mt, bm, h, 0, 0))
            t1 = timeit(lambda: C.moe_gemm(h, w2, ws.sorted_tok, ws.sorted_w, ws.tiles, mt, bm, y, 1, 0))
            print(json.dumps({"tokens": T, "ablate": os.environ.get("NGA_MOE_ABLATE", "0"),
                              "gate_up_us": round(t0, 1), "gate_up_tflops": round(2.0 * M * 2 * F * H / t0 / 1e6, 1),
                              "down_us": round(t1, 1), "down_tflops": round(2.0 * M * F * H / t1 / 1e6, 1)}), flush=True)
            continue
        y = ops.moe_ffn(x, router, w13, w2, k)
        yr = eager(x, router, w13, w2, k)
        rel = ((y.float() - yr.float()).norm() / yr.float().norm()).item()
        t_ours = timeit(lambda: ops.moe_ffn(x, router, w13, w2, k))
        t_eager = timeit(lambda: eager(x, router, w13, w2, k))
        flop = 2.0 * T * k * (2 * F * H + H * F)
        wbytes = min(E, T * k) * 3 * F * H * 2
        print(json.dumps({"tokens": T, "ours_us": round(t_ours, 1), "eager_us": round(t_eager, 1),
                          "speedup": round(t_eager / t_ours, 2),
                          "tflops": round(flop / t_ours / 1e6, 1),
                          "weight_TBps": round(wbytes / t_ours / 1e6, 2), "rel_err": round(rel, 5)}),
              flush=True)


if __name__ == "__main__":
    main()
