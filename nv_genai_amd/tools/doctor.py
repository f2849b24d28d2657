"""Deployment check for one node: ``python -m nv_genai_amd.tools.doctor [--json] [--kernels]``.

Reports what a serving or benchmark run on this node will actually use, before it starts:
- the PyTorch / ROCm / RCCL build and the visible GPUs (name, gfx target, HBM, CU count);
- whether the native libraries load (``_C``: the gfx950 HIP kernels, ``_rt``: the C++ serving
  runtime) and which code objects ``_C`` carries (a build for another target fails at the first
  launch, not at import);
- the kernel-form registry (A/B knobs read once from ``NGA_*``) and every ``NGA_*`` / ``APP_*``
  variable set in the environment;
- the CPU / NUMA placement each local rank would get (``utils/affinity.py``, from the KFD
  topology without starting the HIP runtime) for ``--local-world`` ranks;
- with ``--kernels`` (GPU only): a numerics self-test of the hot kernels against fp32 PyTorch
  (RMSNorm, the decode-shape GEMM with its SwiGLU epilogue, paged decode attention).

Exit status 1 when something a GPU run needs is missing (no ``_C``, no gfx950 code object,
a failed self-test); ``--json`` prints one JSON document instead of the table.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from typing import List


def _gfx_targets(so_path: str) -> List[str]:
    """gfx targets of the code objects bundled in a HIP shared object: the offload-bundle entry
    ids (``hipv4-amdgcn-amd-amdhsa--gfx950``) stored in its ``.hip_fatbin`` section."""
    import re

    if not so_path or not os.path.exists(so_path):
        return []
    with open(so_path, "rb") as f:
        data = f.read()
    return sorted({m.decode() for m in re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", data)})


def collect(local_world: int = 0, run_kernels: bool = False) -> dict:
    rep: dict = {"problems": []}
    # placement first: it reads sysfs only and must not start the HIP runtime
    from ..utils import affinity

    gpus = affinity.visible_gpus()
    n = local_world or max(1, len(gpus))
    rep["placement"] = [affinity.plan(r, n).record() | {"local_rank": r} for r in range(n)] if gpus else []

    import torch

    rep["torch"] = torch.__version__
    rep["hip"] = getattr(torch.version, "hip", None)
    try:
        rep["rccl"] = ".".join(str(x) for x in torch.cuda.nccl.version())
    except Exception:  # noqa: BLE001
        rep["rccl"] = None
    devs = []
    if torch.cuda.is_available():
        for i in range(torch.cuda.device_count()):
            p = torch.cuda.get_device_properties(i)
            devs.append({"index": i, "name": p.name, "arch": getattr(p, "gcnArchName", ""),
                         "hbm_gb": round(p.total_memory / 2 ** 30, 1), "cus": p.multi_processor_count})
    rep["gpus"] = devs
    if devs and not all(d["arch"].startswith("gfx950") for d in devs):
        rep["problems"].append("a visible GPU is not gfx950 (MI355X): the HIP kernels are built for gfx950 only")

    from .. import ops

    rep["native_C"] = ops.have_kernels()
    so = getattr(ops._C, "__file__", "") if ops._C is not None else ""
    rep["native_C_path"] = so
    rep["native_C_targets"] = _gfx_targets(so)
    if not rep["native_C"]:
        rep["problems"].append(f"nv_genai_amd._C does not load: {ops._C_ERR!r} (python -m nv_genai_amd._build)")
    elif rep["native_C_targets"] and "gfx950" not in rep["native_C_targets"]:
        rep["problems"].append(f"_C carries {rep['native_C_targets']}, no gfx950 code object")
    try:
        from .._native import rt

        rep["native_rt"] = True
        rep["native_rt_path"] = getattr(rt, "__file__", "")
    except Exception as e:  # noqa: BLE001
        rep["native_rt"] = False
        rep["problems"].append(f"nv_genai_amd._rt does not load: {e!r}")
    if rep["native_C"]:
        rep["kernel_forms"] = {k: ops.kernel_form(k) for k in ops.KERNEL_FORMS}
    rep["env"] = {k: v for k, v in sorted(os.environ.items()) if k.startswith(("NGA_", "APP_"))
                  or k in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES",
                           "HSA_ENABLE_IPC_MODE_LEGACY", "PYTORCH_ROCM_ARCH")}
    if os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0") != "0":
        rep["problems"].append("HSA_ENABLE_IPC_MODE_LEGACY is not 0: RCCL / IPC tensor sharing needs dmabuf IPC")
    if run_kernels:
        rep["self_test"] = self_test() if devs and rep["native_C"] else {"skipped": "needs a GPU and _C"}
        bad = [k for k, v in rep["self_test"].items() if isinstance(v, dict) and not v.get("ok")]
        if bad:
            rep["problems"].append(f"kernel self-test failed: {bad}")
    return rep


def self_test() -> dict:
    """Hot kernels on cuda:0 against fp32 PyTorch (per-row relative error)."""
    import torch

    from .. import ops

    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    out = {}

    def rel(a, b):
        a, b = a.float(), b.float()
        return float(((a - b).norm(dim=-1) / b.norm(dim=-1).clamp_min(1e-6)).max())

    x = torch.randn(64, 4096, device=dev, dtype=torch.bfloat16, generator=g)
    w = torch.rand(4096, device=dev, dtype=torch.bfloat16, generator=g) + 0.5
    ref = x.float() * torch.rsqrt(x.float().pow(2).mean(-1, keepdim=True) + 1e-5) * w.float()
    e = rel(ops.rmsnorm(x, w, 1e-5), ref)
    out["rmsnorm"] = {"max_row_rel_err": e, "ok": e < 1e-2}

    F, K, M = 2048, 1024, 64
    xw = torch.randn(M, K, device=dev, dtype=torch.bfloat16, generator=g)
    W = torch.randn(2 * F, K, device=dev, dtype=torch.bfloat16, generator=g) * 0.05
    y = xw.float() @ W.float().t()
    ref = torch.nn.functional.silu(y[:, :F]) * y[:, F:]
    e = rel(ops.skinny_gemm(xw, W, 13, 1, 2), ref)
    out["skinny_gemm_swiglu"] = {"max_row_rel_err": e, "ok": e < 2e-2}

    B, L, Hq, Hkv, D = 8, 300, 32, 8, 128
    pages = -(-L // 64)
    kc = torch.randn(B * pages, Hkv, 64, D, device=dev, dtype=torch.bfloat16, generator=g)
    vc = torch.randn(B * pages, Hkv, D, 64, device=dev, dtype=torch.bfloat16, generator=g)
    bt = torch.arange(B * pages, device=dev, dtype=torch.int32).view(B, pages)
    ctx = torch.full((B,), L, device=dev, dtype=torch.int32)
    q = torch.randn(B, Hq * D, device=dev, dtype=torch.bfloat16, generator=g)
    o = ops.decode_attention(q, kc, vc, bt, ctx, Hq, Hkv, L, D ** -0.5)
    # reference: gather the pages back into [B, L, Hkv, D]
    K_ = kc[bt.long()].permute(0, 1, 3, 2, 4).reshape(B, pages * 64, Hkv, D)[:, :L].float()
    V_ = vc[bt.long()].permute(0, 1, 4, 2, 3).reshape(B, pages * 64, Hkv, D)[:, :L].float()
    qf = q.float().view(B, Hkv, Hq // Hkv, D)
    s = torch.einsum("bhgd,blhd->bhgl", qf, K_) * D ** -0.5
    ref = torch.einsum("bhgl,blhd->bhgd", s.softmax(-1), V_).reshape(B, Hq * D)
    e = rel(o, ref)
    out["decode_attention"] = {"max_row_rel_err": e, "ok": e < 2e-2}
    torch.cuda.synchronize()
    return out


def _print(rep: dict) -> None:
    print(f"torch {rep['torch']}  HIP {rep['hip']}  RCCL {rep['rccl']}")
    for d in rep["gpus"] or [{"index": "-", "name": "no GPU visible", "arch": "", "hbm_gb": "", "cus": ""}]:
        print(f"  GPU {d['index']}: {d['name']} {d['arch']} {d['hbm_gb']} GiB {d['cus']} CUs")
    print(f"_C (HIP kernels): {'loaded' if rep['native_C'] else 'MISSING'} {rep.get('native_C_path', '')} "
          f"targets {rep.get('native_C_targets') or '?'}")
    print(f"_rt (C++ runtime): {'loaded' if rep.get('native_rt') else 'MISSING'}")
    if "kernel_forms" in rep:
        print("kernel forms:", " ".join(f"{k}={v}" for k, v in rep["kernel_forms"].items()))
    for k, v in rep["env"].items():
        print(f"  {k}={v}")
    for p in rep["placement"]:
        print(f"  local rank {p['local_rank']}: GPU {p.get('pci_bus_id_sysfs')} NUMA {p['numa_node']} "
              f"cpus {p['cpu_affinity'] or '-'} {p.get('affinity_note', '')}")
    for k, v in (rep.get("self_test") or {}).items():
        print(f"  self-test {k}: {v}")
    print("problems:" if rep["problems"] else "no problems found")
    for p in rep["problems"]:
        print("  -", p)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--json", action="store_true")
    ap.add_argument("--kernels", action="store_true", help="run the GPU kernel self-test")
    ap.add_argument("--local-world", type=int, default=0, help="ranks per node to plan placement for")
    a = ap.parse_args(argv)
    rep = collect(a.local_world, a.kernels)
    if a.json:
        print(json.dumps(rep, indent=1, default=str))
    else:
        _print(rep)
    return 1 if rep["problems"] else 0


if __name__ == "__main__":
    sys.exit(main())
