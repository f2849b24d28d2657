"""Probe: FP8 (OCP e4m3fn) GEMMs through torch._scaled_mm (hipBLASLt) on gfx950 against
bf16, at the Llama-3-8B projection shapes of a mixed step (M = 1536): tensor-wise and
row-wise scales, accuracy vs an fp32 reference and time per GEMM."""
import json

import torch


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
    return a.elapsed_time(b) * 1e3 / iters


def main():
    out = {}
    M = 1536
    f8 = torch.float8_e4m3fn
    for name, (N, K) in {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}.items():
        x = torch.randn(M, K, device="cuda") 
        w = torch.randn(N, K, device="cuda") * 0.02
        ref = x @ w.t()
        xb, wb = x.bfloat16(), w.bfloat16()
        t_bf = timeit(lambda: xb @ wb.t())
        sx = x.abs().amax(1, keepdim=True) / 448.0
        sw = w.abs().amax(1, keepdim=True) / 448.0
        x8 = (x / sx).to(f8)
        w8 = (w / sw).to(f8)
        res = {"bf16_us": round(t_bf, 1), "bf16_TF": round(2 * M * N * K / t_bf / 1e6, 1)}
        try:
            y = torch._scaled_mm(x8, w8.t(), scale_a=sx, scale_b=sw.t(), out_dtype=torch.bfloat16)
            t8 = timeit(lambda: torch._scaled_mm(x8, w8.t(), scale_a=sx, scale_b=sw.t(), out_dtype=torch.bfloat16))
            res.update(rowwise_us=round(t8, 1), rowwise_TF=round(2 * M * N * K / t8 / 1e6, 1),
                       rowwise_rel_err=round(float((y.float() - ref).norm() / ref.norm()), 5))
        except Exception as e:  # noqa: BLE001
            res["rowwise_error"] = repr(e)[:300]
        try:
            st_x = (x.abs().amax() / 448.0).reshape(())
            st_w = (w.abs().amax() / 448.0).reshape(())
            xt, wt = (x / st_x).to(f8), (w / st_w).to(f8)
            y = torch._scaled_mm(xt, wt.t(), scale_a=st_x, scale_b=st_w, out_dtype=torch.bfloat16)
            t8 = timeit(lambda: torch._scaled_mm(xt, wt.t(), scale_a=st_x, scale_b=st_w, out_dtype=torch.bfloat16))
            res.update(tensorwise_us=round(t8, 1), tensorwise_TF=round(2 * M * N * K / t8 / 1e6, 1),
                       tensorwise_rel_err=round(float((y.float() - ref).norm() / ref.norm()), 5))
        except Exception as e:  # noqa: BLE001
            res["tensorwise_error"] = repr(e)[:300]
        res["bf16_rel_err"] = round(float(((xb @ wb.t()).float() - ref).norm() / ref.norm()), 5)
        out[name] = res
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
