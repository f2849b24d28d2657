#!/bin/bash
# Round 4: skinny configs with more waves per CU (2-3 blocks per CU: cfg 17-19) vs the table's
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r4_skinny_waves; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "skinny_gemm_every_cfg" > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -1 $O/test.txt
timeout -k 10 400 python -u benchmarks/skinny_gemm.py --ms 64,128,256 --shapes o,qkv,down,gate_up --cfgs 1,2,3,11,13,16,17,18,19 --all > $O/sweep.jsonl 2>&1 || { tail -20 $O/sweep.jsonl; exit 1; }
grep '"lib_us"' $O/sweep.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); b=r['best_gemm']; print(r['shape'], r['M'], 'lib', r['lib_us'], 'best', b['cfg'], b['split'], b['gemm_us'], b['total_us'])"
python3 - <<'PY'
import json
best = {}
for l in open("gpurun_out/r4_skinny_waves/sweep.jsonl"):
    if not l.startswith("{") or '"lib_us"' in l:
        continue
    r = json.loads(l)
    if "cfg" not in r:
        continue
    k = (r.get("shape"), r.get("M"), r["cfg"])
    t = r.get("total_us", r.get("gemm_us"))
    if t is not None and (k not in best or t < best[k]):
        best[k] = t
for k in sorted(best):
    if k[2] >= 17:
        print("new cfg", k, best[k])
PY
