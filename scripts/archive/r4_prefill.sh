#!/bin/bash
# Round 4: prefill attention — 8-wave shared-tile form (impl 5) vs the shipped forms
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r4_prefill; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "prefill_attention" > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -2 $O/test.txt
timeout -k 10 300 python -u benchmarks/kernel_bench.py --only prefill > $O/kb_prefill.json 2> $O/kb_prefill.err || { tail -20 $O/kb_prefill.err; exit 1; }
python3 - <<'PY'
import json
d=json.load(open("gpurun_out/r4_prefill/kb_prefill.json"))
for k,v in d.items():
    if k.startswith("prefill"):
        print(k, {t: (x["us"], x["TFLOPs"]) for t,x in v.items()})
PY
