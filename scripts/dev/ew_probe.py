"""Elementwise kernels of the mixed step at its token counts: silu_mul (gate|up -> SwiGLU, F
14,336) and add + RMSNorm (4,096 wide); device time per call and the HBM-equivalent rate.
(profiles/r6_ew/probe.json also holds a row-blocked silu_mul variant, v1, measured against the
shipped flat grid-stride kernel, v0, and not kept: equal within 3 %.)"""
import json

import torch

from nv_genai_amd import ops
from nv_genai_amd.ops import reference as ref


def timeit(fn, n=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


def main():
    dev = torch.device("cuda:0")
    F = 14336
    out = {}
    for M in (256, 1426, 2048, 4352):
        x = (torch.randn(M, 2 * F, device=dev) * 2).to(torch.bfloat16)
        o = torch.empty(M, F, dtype=torch.bfloat16, device=dev)
        want = ref.silu_mul(x.float()).to(torch.bfloat16).float()
        us = timeit(lambda: ops.silu_mul(x, out=o))
        err = ((o.float() - want).abs().max() / want.abs().max()).item()
        row = {"us": round(us, 2), "TBps": round(M * F * 6 / us / 1e6, 2), "max_rel_err": err}
        out[f"silu_mul_{M}x{F}"] = row
        print(json.dumps({f"silu_mul_{M}x{F}": row}), flush=True)
    w = torch.randn(4096, device=dev).to(torch.bfloat16)
    for M in (256, 1426, 4352):
        r = torch.randn(M, 4096, device=dev).to(torch.bfloat16)
        d = torch.randn(M, 4096, device=dev).to(torch.bfloat16)
        o = torch.empty_like(r)
        us = timeit(lambda: ops.add_rmsnorm(r, d, w, 1e-5, out=o))
        out[f"add_rmsnorm_{M}x4096"] = {"us": round(us, 2), "TBps": round(M * 4096 * 8 / us / 1e6, 2)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
