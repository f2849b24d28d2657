"""Re-tune selected projection GEMM shapes with cold operands and merge them into a TunableOp
table.

The shipped table was tuned with the same weight tensor on every timing iteration, so a
small-M GEMM whose weights fit the 256 MB MALL was timed warm. In a forward pass every layer
streams its own weights from HBM, so the fastest warm solution need not be the fastest cold
one. Here TunableOp's rotating buffer (larger than the MALL) gives every iteration fresh
operands.

    python scripts/retune_cold.py --ms 256 --rotating-mb 1024 --out gpurun_out/cold/gemm_cold.csv
    python scripts/retune_cold.py --merge --out gpurun_out/cold/gemm_cold.csv   # TunableOp writes at exit
"""
import argparse
import csv
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.cuda.tunable as tn  # noqa: E402

from nv_genai_amd.models.config import llama_config  # noqa: E402
from nv_genai_amd.ops.gemm_tuning import llm_gemm_shapes  # noqa: E402


def merge(base: str, fresh: str, out: str) -> int:
    """Rows of ``fresh`` replace the rows of ``base`` with the same (op, shape) key; returns
    the number of replaced or added rows."""
    with open(base) as f:
        rows = [r for r in csv.reader(f)]
    with open(fresh) as f:
        new = {(r[0], r[1]): r for r in csv.reader(f) if r and not r[0].startswith("Validator")}
    seen, n = set(), 0
    merged = []
    for r in rows:
        k = (r[0], r[1]) if len(r) > 1 else None
        if k in new:
            merged.append(new[k])
            seen.add(k)
            n += 1
        else:
            merged.append(r)
    for k, r in new.items():
        if k not in seen:
            merged.append(r)
            n += 1
    with open(out, "w", newline="") as f:
        csv.writer(f, lineterminator="\n").writerows(merged)
    return n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--ms", default="256")
    ap.add_argument("--rotating-mb", type=int, default=1024)
    ap.add_argument("--base", default="nv_genai_amd/assets/tunableop/gemm_gfx950.csv")
    ap.add_argument("--out", required=True)
    ap.add_argument("--max-ms", type=int, default=30)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--merge", action="store_true", help="only merge OUT.fresh.csv (written by a tuning run) into BASE")
    args = ap.parse_args()
    if args.merge:
        n = merge(args.base, args.out + ".fresh.csv", args.out)
        print(f"merged {n} cold-tuned rows into {args.out}", flush=True)
        return
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    fresh = args.out + ".fresh.csv"
    if os.path.exists(fresh):
        os.remove(fresh)
    cfg = llama_config(args.model)
    ms = [int(x) for x in args.ms.split(",") if x]
    shapes = [s for s in llm_gemm_shapes(cfg, 1, [], ms)]
    tn.enable(True)
    tn.tuning_enable(True)
    tn.set_filename(os.path.abspath(fresh), insert_device_ordinal=False)
    tn.set_max_tuning_duration(args.max_ms)
    tn.set_max_tuning_iterations(args.iters)
    tn.set_rotating_buffer_size(args.rotating_mb)
    dev = torch.device("cuda:0")
    t0 = time.time()
    for i, (m, n, k) in enumerate(shapes):
        w = torch.randn(n, k, device=dev, dtype=torch.bfloat16) * 0.02
        x = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
        y = x @ w.t()
        torch.cuda.synchronize()
        print(f"[{i + 1}/{len(shapes)}] M={m} N={n} K={k} {time.time() - t0:.0f}s", flush=True)
        del x, y, w
    print("tuned rows are written to", fresh, "at exit; merge with --merge", flush=True)


if __name__ == "__main__":
    main()
