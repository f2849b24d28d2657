#!/bin/bash
# Round 4: headline vs NGA_PF_SEQ_MIN (large prefills after the decode attention), interleaved
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r4_pfseq_ab; mkdir -p $O
i=0
for v in ${VALS:-384 192 384 192}; do
  i=$((i+1))
  NGA_PF_SEQ_MIN=$v timeout -k 10 420 python -u bench.py --steps 10 --warmup 3 > $O/bench_${i}_$v.json 2> $O/bench_${i}_$v.err || { tail -20 $O/bench_${i}_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_${i}_$v.json'));print('pf_seq_min $v', d['value'], d['p50_latency_ms'], d['p50_ttft_ms'])"
done
