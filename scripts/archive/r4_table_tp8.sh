#!/bin/bash
# Round 4: decode-shape GEMM table for the llama3-70b TP=8 rank shapes (merged into the shipped table)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r4_table_tp8; mkdir -p $O
cp nv_genai_amd/assets/skinny_gemm_gfx950.json $O/base.json
timeout -k 10 900 python -u benchmarks/skinny_table.py --model llama3-70b --tp 8 --merge $O/base.json --out $O/skinny_gemm_gfx950.json > $O/table.jsonl 2>&1 || { tail -20 $O/table.jsonl; exit 1; }
python3 -c "
import json
for l in open('$O/table.jsonl'):
    if l.startswith('{'):
        r=json.loads(l); print(r['shape'], r['N'], r['K'], r['M'], 'lib', r['lib_us'], 'best', r.get('cfg'), r.get('split'), r.get('best_us'), r.get('speedup'))"
