"""Probe torch._grouped_mm on this ROCm build: correctness vs per-expert matmul and speed at
Mixtral prefill sizes (1,536 tokens, top-2, 8 experts, H 4096, F 14336)."""
import json
import time

import torch

dev = "cuda"
torch.manual_seed(0)
E, H, F = 8, 4096, 14336
res = {}
for T in (256, 1536, 4096):
    rows = 2 * T
    cnt = torch.distributions.Multinomial(rows, torch.ones(E)).sample().long()
    offs = torch.cumsum(cnt, 0).to(torch.int32).to(dev)
    a = torch.randn(rows, H, device=dev, dtype=torch.bfloat16)
    w = torch.randn(E, 2 * F, H, device=dev, dtype=torch.bfloat16) * 0.02  # [E, N, K] as nn.Linear
    wt = w.transpose(1, 2)  # [E, K, N] view
    try:
        out = torch._grouped_mm(a, wt, offs=offs)
    except Exception as e:  # noqa: BLE001
        res[f"T{T}"] = {"error": repr(e)[:300]}
        continue
    ref = torch.empty_like(out)
    s = 0
    for e_, c in enumerate(cnt.tolist()):
        ref[s:s + c] = a[s:s + c] @ wt[e_]
        s += c
    err = (out.float() - ref.float()).abs().max().item()

    def timeit(fn, it=20):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(it):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / it * 1e6

    us = timeit(lambda: torch._grouped_mm(a, wt, offs=offs))
    us_loop = timeit(lambda: [a[:c] @ wt[i] for i, c in enumerate(cnt.tolist())])
    fl = 2 * rows * H * 2 * F
    res[f"T{T}"] = {"max_err": err, "grouped_us": round(us, 1), "grouped_tflops": round(fl / us / 1e6, 1),
                    "loop_us": round(us_loop, 1), "loop_tflops": round(fl / us_loop / 1e6, 1)}
    print(json.dumps({f"T{T}": res[f"T{T}"]}), flush=True)
print(json.dumps(res))
