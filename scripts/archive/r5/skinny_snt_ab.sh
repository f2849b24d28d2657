#!/bin/bash
# Round 5: skinny_snt (decode-shape GEMM fp32 K-split slabs: 1 non-temporal stores, 2 also
# non-temporal loads in their consumers): numerics, decode step interleaved 0/1/2 x 2, headline
# (8 steps / 2 warm-up) interleaved 0/2 x 2
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/r5_skinny_snt
mkdir -p $out
timeout -k 10 200 python -u -m pytest -q -p no:cacheprovider --timeout 150 --timeout-method thread tests/test_kernels_gpu.py -k "splitk or nontemporal or rope" > $out/tests.txt 2>&1 || { tail -30 $out/tests.txt; exit 1; }
tail -1 $out/tests.txt
for r in 1 2; do
  for v in 0 1 2; do
    NGA_SKINNY_SNT=$v timeout -k 10 300 python benchmarks/decode_step.py --batch 256 --ctx 1400 --steps 48 > $out/decode_${v}_$r.json 2> $out/decode_${v}_$r.err || { tail -5 $out/decode_${v}_$r.err; exit 1; }
    echo "decode snt $v round $r $(python3 -c "import json;d=json.load(open('$out/decode_${v}_$r.json'));print(d['replay_ms'], d['step_ms'])")"
  done
done
for rv in "0 1" "2 1" "0 2" "2 2"; do
  set -- $rv; v=$1; r=$2
  NGA_SKINNY_SNT=$v timeout -k 10 300 python bench.py --steps 8 --warmup 2 > $out/bench_${v}_$r.json 2> $out/bench_${v}_$r.err || { tail -5 $out/bench_${v}_$r.err; exit 1; }
  echo "bench snt $v round $r $(python3 -c "import json;d=json.load(open('$out/bench_${v}_$r.json'));print(d['value'], d['p50_latency_ms'])")"
done
