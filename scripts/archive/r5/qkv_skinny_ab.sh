#!/bin/bash
# Round 5: q/k/v at M = 192-256 on the decode-shape kernel (nt weight DMA, K-split slabs summed
# by the RoPE kernel) instead of the library GEMM the isolated table picked (34.5 vs 35.5 us):
# does the in-step picture differ? Variant table = shipped table with those three entries
# replaced; decode step interleaved x 2, headline (8 steps / 2 warm-up) interleaved x 2
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/r5_qkv_skinny
mkdir -p $out
python3 - <<'PY'
import json
t = json.load(open("nv_genai_amd/assets/skinny_gemm_gfx950.json"))
t["table"]["6144x4096"]["by_m"].update({"192": [2, 3], "224": [1, 2], "256": [1, 2]})
json.dump(t, open("gpurun_out/r5_qkv_skinny/table_qkv_skinny.json", "w"))
PY
tab=$PWD/$out/table_qkv_skinny.json
timeout -k 10 200 python -u -m pytest -q -p no:cacheprovider --timeout 150 --timeout-method thread tests/test_kernels_gpu.py -k "skinny_table or rope_cache_from_splitk" > $out/tests.txt 2>&1 || { tail -30 $out/tests.txt; exit 1; }
tail -1 $out/tests.txt
for r in 1 2; do
  for v in lib sk; do
    if [ $v = sk ]; then export NGA_SKINNY_TABLE=$tab; else unset NGA_SKINNY_TABLE; fi
    timeout -k 10 300 python benchmarks/decode_step.py --batch 256 --ctx 1400 --steps 48 > $out/decode_${v}_$r.json 2> $out/decode_${v}_$r.err || { tail -5 $out/decode_${v}_$r.err; exit 1; }
    echo "decode qkv $v round $r $(python3 -c "import json;d=json.load(open('$out/decode_${v}_$r.json'));print(d['replay_ms'], d['step_ms'])")"
  done
done
for r in 1 2; do
  for v in lib sk; do
    if [ $v = sk ]; then export NGA_SKINNY_TABLE=$tab; else unset NGA_SKINNY_TABLE; fi
    timeout -k 10 300 python bench.py --steps 8 --warmup 2 > $out/bench_${v}_$r.json 2> $out/bench_${v}_$r.err || { tail -5 $out/bench_${v}_$r.err; exit 1; }
    echo "bench qkv $v round $r $(python3 -c "import json;d=json.load(open('$out/bench_${v}_$r.json'));print(d['value'], d['p50_latency_ms'])")"
  done
done
