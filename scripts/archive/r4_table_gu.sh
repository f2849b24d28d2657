#!/bin/bash
# Round 4: gate/up re-measured with K-split slabs + the SwiGLU consumer (merged into the shipped table)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r4_table_gu; mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "splitk" > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -1 $O/test.txt
cp nv_genai_amd/assets/skinny_gemm_gfx950.json $O/base.json
timeout -k 10 600 python -u benchmarks/skinny_table.py --model llama3-8b --shapes gate_up --merge $O/base.json --out $O/skinny_gemm_gfx950.json > $O/table.jsonl 2>&1 || { tail -20 $O/table.jsonl; exit 1; }
python3 -c "
import json
for l in open('$O/table.jsonl'):
    if l.startswith('{'):
        r=json.loads(l); print(r['shape'], r['M'], 'lib', r['lib_us'], 'best', r.get('cfg'), r.get('split'), r.get('best_us'), r.get('speedup'))"
