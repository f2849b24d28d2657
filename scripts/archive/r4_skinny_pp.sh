#!/bin/bash
# Round 4: ping-pong schedule for the decode-shape GEMM (cfg 17-19): numerics of every cfg, then
# a sweep against the shipped configurations
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r4_skinny_pp; mkdir -p $O
timeout -k 10 180 python -u -m pytest -x -q --timeout 90 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "skinny_gemm_every_cfg" > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -1 $O/test.txt
timeout -k 10 400 python -u benchmarks/skinny_gemm.py --ms 64,128,256 --shapes o,qkv,down,gate_up --cfgs 1,2,3,13,16,17,18,19 --all > $O/sweep.jsonl 2>&1 || { tail -20 $O/sweep.jsonl; exit 1; }
python3 - <<'PY'
import json
best = {}
rows = []
for l in open("gpurun_out/r4_skinny_pp/sweep.jsonl"):
    if not l.startswith("{"):
        continue
    r = json.loads(l)
    if "lib_us" in r:
        rows.append(r)
        continue
    k = (r["shape"], r["M"], r["cfg"] >= 17)
    if k not in best or r["total_us"] < best[k][0]:
        best[k] = (r["total_us"], r["cfg"], r["split"], r["gemm_us"])
for r in rows:
    a = best.get((r["shape"], r["M"], False)); b = best.get((r["shape"], r["M"], True))
    print(r["shape"], r["M"], "lib", r["lib_us"], "shipped-best", a, "ping-pong-best", b)
PY
