#!/bin/bash
# Round 4: selection table rows for the mixed-step buckets (768-4096 rows)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r4_table_large; mkdir -p $O
timeout -k 10 1000 python -u benchmarks/skinny_table.py --ms 768,1024,1280,1536,1792,2048,2304,2560,2816,3072,3328,3584,3840,4096 \
  --merge nv_genai_amd/assets/skinny_gemm_gfx950.json --out $O/skinny_gemm_gfx950.json > $O/table.jsonl 2>&1 || { tail -20 $O/table.jsonl; exit 1; }
python3 -c "
import json
for l in open('$O/table.jsonl'):
    if l.startswith('{'):
        r=json.loads(l); print(r['shape'], r['M'], 'lib', r['lib_us'], 'best', r.get('cfg'), r.get('split'), r.get('best_us'), r.get('speedup'))"
