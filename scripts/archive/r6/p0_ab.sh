#!/bin/bash
# Round 6: decode attention with each sequence's first KV page loaded with the default cache
# policy (shared prompt-template page, L2 hits) vs nt everywhere: numerics, then interleaved
# headline (8 steps) and the decode step
set -o pipefail
cd "$(dirname "$0")/../../.."
out=gpurun_out/${1:-r6_p0}
mkdir -p $out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "decode_attention" -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for i in 1 2; do
  for a in 4 2; do
    NGA_DECODE_DMA_AUX=$a timeout -k 10 400 python bench.py --steps 8 --warmup 2 > $out/bench_aux${a}_$i.json 2> $out/bench_aux${a}_$i.err || { tail -20 $out/bench_aux${a}_$i.err; exit 1; }
    python -c "import json;d=json.load(open('$out/bench_aux${a}_$i.json'));print('aux=$a', d['value'], d['p50_latency_ms'], d['prefix_cache']['hit_share'])"
  done
done
for a in 4 2; do
  NGA_DECODE_DMA_AUX=$a timeout -k 10 300 python benchmarks/decode_step.py --batch 256 --ctx 1400 --steps 16 > $out/decode_aux$a.json 2> $out/decode_aux$a.err || { tail -20 $out/decode_aux$a.err; exit 1; }
  echo "aux=$a $(tail -1 $out/decode_aux$a.json)"
done
