"""Run one skinny-GEMM configuration in a loop (a target for rocprofv3 counter passes):
``--shape o --m 256 --cfg 1 --split 4``; weights rotate over copies past the MALL."""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from nv_genai_amd import ops  # noqa: E402

SHAPES = {"qkv": (6144, 4096, 0), "o": (4096, 4096, 0), "gate_up": (28672, 4096, 2),
          "down": (4096, 14336, 0), "lm_head": (128256, 4096, 0)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="o")
    ap.add_argument("--m", type=int, default=256)
    ap.add_argument("--cfg", type=int, default=1)
    ap.add_argument("--split", type=int, default=4)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--lib", action="store_true", help="the library GEMM instead")
    ap.add_argument("--krot", type=int, default=0)
    ap.add_argument("--wpack", action="store_true")
    ap.add_argument("--tuned", action="store_true", help="library GEMM with the shipped TunableOp table")
    a = ap.parse_args()
    if a.tuned:
        from nv_genai_amd.ops.gemm_tuning import use_tuned_gemms

        use_tuned_gemms()
    N, K, epi = SHAPES[a.shape]
    n_rot = max(2, math.ceil(640e6 / (N * K * 2)))
    dev = torch.device("cuda")
    Ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(n_rot)]
    x = torch.randn(a.m, K, device=dev, dtype=torch.bfloat16)
    e = epi if a.split == 1 else 1
    out = (torch.empty(a.split, a.m, N, device=dev) if e == 1 else
           torch.empty(a.m, N // 2 if e == 2 else N, device=dev, dtype=torch.bfloat16))
    C = ops.kernels()
    nout = 0
    if a.wpack:
        Ws = [ops.pack_weight(w, C.skinny_cfg(a.cfg)[0], epi) for w in Ws]
        nout = N // 2 if epi == 2 else N
    for i in range(a.iters):
        if a.lib:
            x @ Ws[i % n_rot].t()
        else:
            C.skinny_gemm(out, x, Ws[i % n_rot], e, a.split, a.cfg, a.krot, 1 if a.wpack else 0, nout, 0, 0)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
