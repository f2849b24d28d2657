#!/bin/bash
# Round 4: decode-shape GEMM table for llama3-70b (TP=1 shapes, merged), then the 70B agent
# workload on one GPU with the kernel off / on (interleaved)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r4_agent70b; mkdir -p $O
cp nv_genai_amd/assets/skinny_gemm_gfx950.json $O/base.json
if [ -z "$SKIP_TABLE" ]; then
  timeout -k 10 900 python -u benchmarks/skinny_table.py --model llama3-70b --ms 16,32,64,96,128,160,192,256 --merge $O/base.json --out $O/skinny_gemm_gfx950.json > $O/table.jsonl 2>&1 || { tail -20 $O/table.jsonl; exit 1; }
  cp $O/skinny_gemm_gfx950.json nv_genai_amd/assets/skinny_gemm_gfx950.json
  python3 -c "
import json
for l in open('$O/table.jsonl'):
    if l.startswith('{'):
        r=json.loads(l); print(r['shape'], r['M'], 'lib', r['lib_us'], 'best', r.get('cfg'), r.get('split'), r.get('best_us'), r.get('speedup'))"
fi
for v in ${ARMS:-0 1}; do
  NGA_SKINNY=$v timeout -k 10 600 python -u benchmarks/agent_tp.py --model llama3-70b --index-size 10000000 --out $O/agent_sk$v.json > $O/agent_sk$v.log 2>&1 || { tail -20 $O/agent_sk$v.log; exit 1; }
  echo "skinny $v: $(cat $O/agent_sk$v.json)"
done
