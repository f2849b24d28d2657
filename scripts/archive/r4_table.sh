#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r4_table; mkdir -p $O
timeout -k 10 900 python -u benchmarks/skinny_table.py --model llama3-8b --out $O/skinny_gemm_gfx950.json > $O/table.jsonl 2>&1 || { tail -20 $O/table.jsonl; exit 1; }
python3 -c "
import json
for l in open('$O/table.jsonl'):
    if l.startswith('{'):
        r=json.loads(l); print(r['shape'], r['M'], 'lib', r['lib_us'], 'best', r.get('cfg'), r.get('split'), r.get('best_us'), r.get('speedup'))"
