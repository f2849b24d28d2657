#!/bin/bash
# Round 5: decode_dma_aux (cache policy of the LDS-DMA decode kernel's KV loads: 2 nt, 0 default) A/B where it
# matters: the decode step interleaved 2/0 x 2, then the headline (8 steps / 2 warm-up)
# interleaved 2/0 x 2
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/r5_dma_aux
mkdir -p $out
timeout -k 10 200 python -u -m pytest -q -p no:cacheprovider --timeout 150 --timeout-method thread tests/test_kernels_gpu.py -k "decode_attention" > $out/tests.txt 2>&1 || { tail -30 $out/tests.txt; exit 1; }
tail -1 $out/tests.txt
for r in 1 2; do
  for v in 2 0; do
    NGA_DECODE_DMA_AUX=$v timeout -k 10 300 python benchmarks/decode_step.py --batch 256 --ctx 1400 --steps 48 > $out/decode_${v}_$r.json 2> $out/decode_${v}_$r.err || { tail -5 $out/decode_${v}_$r.err; exit 1; }
    echo "decode aux $v round $r $(python3 -c "import json;d=json.load(open('$out/decode_${v}_$r.json'));print(d['replay_ms'], d['step_ms'])")"
  done
done
for rv in "2 1" "0 1" "2 2" "0 2"; do
  set -- $rv; v=$1; r=$2
  NGA_DECODE_DMA_AUX=$v timeout -k 10 300 python bench.py --steps 8 --warmup 2 > $out/bench_${v}_$r.json 2> $out/bench_${v}_$r.err || { tail -5 $out/bench_${v}_$r.err; exit 1; }
  echo "bench aux $v round $r $(python3 -c "import json;d=json.load(open('$out/bench_${v}_$r.json'));print(d['value'], d['p50_latency_ms'])")"
done
