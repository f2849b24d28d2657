"""Tune the LLM's projection GEMMs on an MI355X and write the TunableOp table that
``nv_genai_amd.ops.gemm_tuning.use_tuned_gemms`` loads (see that module's docstring).

    python scripts/tune_gemms.py --model llama3-8b --out nv_genai_amd/assets/tunableop/gemm_gfx950.csv
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.cuda.tunable as tn  # noqa: E402

from nv_genai_amd.models.config import llama_config  # noqa: E402
from nv_genai_amd.ops.gemm_tuning import llm_gemm_shapes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--decode", default="1,2,4,8,16,24,32,48,64,96,128,160,192,224,256")
    ap.add_argument("--prefill", default="32768,16384")
    ap.add_argument("--out", default="nv_genai_amd/assets/tunableop/gemm_gfx950.csv")
    ap.add_argument("--max-ms", type=int, default=20)
    ap.add_argument("--iters", type=int, default=40)
    args = ap.parse_args()
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    cfg = llama_config(args.model)
    shapes = llm_gemm_shapes(cfg, args.tp, [int(x) for x in args.decode.split(",") if x],
                             [int(x) for x in args.prefill.split(",") if x])
    tn.enable(True)
    tn.tuning_enable(True)
    tn.set_filename(os.path.abspath(args.out), insert_device_ordinal=False)
    if os.path.exists(args.out):
        tn.read_file(args.out)
    tn.set_max_tuning_duration(args.max_ms)
    tn.set_max_tuning_iterations(args.iters)
    dev = torch.device("cuda:0")
    ws = {}
    t0 = time.time()
    for i, (m, n, k) in enumerate(shapes):
        if (n, k) not in ws:
            ws[(n, k)] = torch.randn(n, k, device=dev, dtype=torch.bfloat16) * 0.02
        x = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
        y = x @ ws[(n, k)].t()
        torch.cuda.synchronize()
        print(f"[{i + 1}/{len(shapes)}] M={m} N={n} K={k} {time.time() - t0:.0f}s", flush=True)
        del x, y
    print("results are written to", args.out, "at exit", flush=True)


if __name__ == "__main__":
    main()
