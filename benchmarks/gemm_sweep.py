"""Time the Llama-3-8B projection GEMMs (x @ W^T, bf16) over a sweep of token counts M with
the library default and (optionally) the shipped TunableOp table; prints PFLOP/s."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="256,512,1024,1452,1536,2048,3072,4096,8192,16384,32768")
    ap.add_argument("--tuned", action="store_true")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    if a.tuned:
        from nv_genai_amd.ops.gemm_tuning import use_tuned_gemms
        print("table loaded:", use_tuned_gemms(), flush=True)
    dev = torch.device("cuda")
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
    W = {k: torch.randn(n, kk, device=dev, dtype=torch.bfloat16) * 0.02 for k, (n, kk) in shapes.items()}
    out = []
    for m in [int(x) for x in a.ms.split(",")]:
        row = {"M": m}
        tot_t, tot_f = 0.0, 0.0
        for k, w in W.items():
            x = torch.randn(m, w.shape[1], device=dev, dtype=torch.bfloat16)
            for _ in range(3):
                x @ w.t()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                x @ w.t()
            e1.record()
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1) / a.iters / 1e3
            f = 2.0 * m * w.shape[0] * w.shape[1]
            row[k] = round(f / t / 1e15, 3)
            row[k + "_us"] = round(t * 1e6, 1)
            row[k + "_TBps"] = round((w.numel() + x.numel() + m * w.shape[0]) * 2 / t / 1e12, 2)
            tot_t += t
            tot_f += f
        row["layer_us"] = round(tot_t * 1e6, 1)
        row["layer_PF"] = round(tot_f / tot_t / 1e15, 3)
        print(json.dumps(row), flush=True)
        out.append(row)


if __name__ == "__main__":
    main()
