"""Weight-streaming GEMV (csrc/kernels/gemv.hip) vs the decode-shape GEMM table's pick and the
library GEMM at M = 1..4 on the Llama-3-8B projection shapes. Weights rotate over copies past
the 256 MB Infinity Cache (a decode step streams every layer's weights once). One JSON line
per (shape, M) with microseconds and the weight-stream rate of the GEMV.

Usage: ``python benchmarks/gemv_bench.py [--model llama3-8b] [--ms 1,2,4]``.
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


def timeit(fn, n_rot, iters=30):
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
    ap.add_argument("--ms", default="1,2,3,4")
    a = ap.parse_args()
    use_tuned_gemms()
    cfg = llama_config(a.model)
    H, F, D = cfg.hidden, cfg.ffn, cfg.head_dim
    shapes = {"qkv": ((cfg.heads + 2 * cfg.kv_heads) * D, H, 0), "o": (H, cfg.heads * D, 0),
              "gate_up": (2 * F, H, 2), "down": (H, F, 0), "lm_head": (cfg.vocab_size, H, 1)}
    dev = torch.device("cuda")
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    tab = ops.skinny.table()
    for name, (N, K, epi) in shapes.items():
        n_rot = max(2, math.ceil(640e6 / (N * K * 2)))
        Ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16, generator=g) * 0.02 for _ in range(n_rot)]
        for M in [int(m) for m in a.ms.split(",")]:
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16, generator=g)
            ref = x.float() @ Ws[0].float().t()
            if epi == 2:
                ref = torch.nn.functional.silu(ref[:, : N // 2]) * ref[:, N // 2:]
            y = ops.gemv(x, Ws[0], epi).float()
            err = float(((y - ref).norm(dim=1) / ref.norm(dim=1).clamp_min(1e-6)).max())
            gv = timeit(lambda i: ops.gemv(x, Ws[i], epi), n_rot)
            if epi == 2:
                lib = timeit(lambda i: ops.silu_mul(x @ Ws[i].t()), n_rot)
            elif epi == 1:
                lib = timeit(lambda i: (x @ Ws[i].t()).float(), n_rot)
            else:
                lib = timeit(lambda i: x @ Ws[i].t(), n_rot)
            pk = tab.pick(N, K, M)
            sk = None
            if pk is not None:
                c, s = pk
                if epi == 2:
                    sk = timeit(lambda i: ops.skinny_gemm(x, Ws[i], c, 1, 2) if s == 1 else
                                ops.splitk_swiglu(ops.skinny_gemm(x, Ws[i], c, s, 1)), n_rot)
                elif s == 1:
                    sk = timeit(lambda i: ops.skinny_gemm(x, Ws[i], c, 1, 1 if epi == 1 else 0), n_rot)
                else:
                    sk = timeit(lambda i: ops.splitk_reduce(ops.skinny_gemm(x, Ws[i], c, s, 1)), n_rot)
            print(json.dumps({"shape": name, "N": N, "K": K, "M": M, "gemv_us": round(gv, 2),
                              "skinny_us": round(sk, 2) if sk else None, "lib_us": round(lib, 2),
                              "gemv_TBps": round(N * K * 2 / gv / 1e6, 2), "rel_err": round(err, 5)}), flush=True)
        del Ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
