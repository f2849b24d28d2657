"""Does a step's H2D upload block the host while the stream is busy, and does a scatter kernel
reading mapped (fine-grained) host memory avoid it?

For each form, a ~20 ms sleep kernel is queued first, then the upload is issued and the HOST
time of the issuing call is measured (an async call returns in microseconds; a call that waits
for the stream returns after the sleep). Then the device time of back-to-back uploads, and the
data check of the mapped form.
"""
import json
import time

import torch

from nv_genai_amd import ops


def main():
    dev = torch.device("cuda:0")
    C = ops.kernels()
    nb = 24 * 1024
    out = {"bytes": nb}
    h_pin = torch.empty(nb, dtype=torch.uint8, pin_memory=True)
    h_map = C.host_staging(nb)
    d_stage = torch.empty(nb, dtype=torch.uint8, device=dev)
    dsts = [torch.zeros(n, dtype=torch.uint8, device=dev) for n in (4096, 8192, 8192, 4096)]
    offs, o = [], 0
    for d in dsts:
        offs.append(o)
        o += d.numel()
    dst_ptrs = [d.data_ptr() for d in dsts]
    sizes = [d.numel() for d in dsts]
    g = torch.Generator().manual_seed(0)
    src = torch.randint(0, 255, (nb,), generator=g, dtype=torch.uint8)
    h_pin.copy_(src)
    h_map.copy_(src)

    def packed():   # the first packed-upload form: one async copy into device staging + the scatter
        d_stage.copy_(h_pin, non_blocking=True)
        C.scatter_segments(d_stage, dst_ptrs, offs, sizes)

    def mapped():
        C.scatter_host(h_map, 0, dst_ptrs, offs, sizes)

    def plain_copy():
        d_stage.copy_(h_pin, non_blocking=True)

    def kernel_only():
        C.scatter_segments(d_stage, dst_ptrs, offs, sizes)

    forms = {"copy_then_scatter": packed, "mapped_scatter": mapped, "copy_non_blocking": plain_copy,
             "scatter_kernel_only": kernel_only}
    for name, fn in forms.items():
        fn()
        torch.cuda.synchronize()
        host_us = []
        for _ in range(5):
            torch.cuda._sleep(40_000_000)       # ~20 ms of GPU time queued ahead
            t0 = time.perf_counter()
            fn()
            host_us.append((time.perf_counter() - t0) * 1e6)
            torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(200):
            fn()
        e1.record()
        torch.cuda.synchronize()
        t_sleep0 = time.perf_counter()
        torch.cuda._sleep(40_000_000)
        torch.cuda.synchronize()
        sleep_ms = (time.perf_counter() - t_sleep0) * 1e3
        out[name] = {"host_us_behind_busy_stream": [round(x, 1) for x in host_us],
                     "device_us_per_call": round(e0.elapsed_time(e1) * 1e3 / 200, 2),
                     "sleep_ms": round(sleep_ms, 2)}
        print(json.dumps({name: out[name]}), flush=True)
    # data check of the mapped form: rewrite the host buffer, scatter, compare
    src2 = torch.randint(0, 255, (nb,), generator=g, dtype=torch.uint8)
    h_map.copy_(src2)
    mapped()
    torch.cuda.synchronize()
    ok = all(torch.equal(d.cpu(), src2[offs[i]:offs[i] + sizes[i]]) for i, d in enumerate(dsts))
    out["mapped_data_ok"] = ok
    print(json.dumps(out), flush=True)
    assert ok


if __name__ == "__main__":
    main()
