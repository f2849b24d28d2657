#!/usr/bin/env bash
# Decode attention LDS-DMA kernel: numerics tests, then kernel A/B against the register-load
# kernel (NGA_DECODE_DMA=0), then the headline bench.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${1:-r3_dma}"
mkdir -p "$O"
cd "$R"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "decode" --timeout 120 --timeout-method thread > "$O/test_decode.log" 2>&1 || { tail -30 "$O/test_decode.log"; exit 1; }
tail -2 "$O/test_decode.log"
timeout -k 10 300 python benchmarks/kernel_bench.py --only decode > "$O/kb_decode_dma.json" 2> "$O/kb.err" || exit 1
NGA_DECODE_DMA=0 timeout -k 10 300 python benchmarks/kernel_bench.py --only decode > "$O/kb_decode_reg.json" 2>> "$O/kb.err" || exit 1
[ -n "${SKIP_BENCH:-}" ] && exit 0
for r in 1 2; do
  timeout -k 10 420 python bench.py --steps 5 --warmup 2 > "$O/bench_dma_$r.json" 2> "$O/bench_dma_$r.err" || exit 1
  NGA_DECODE_DMA=0 timeout -k 10 420 python bench.py --steps 5 --warmup 2 > "$O/bench_reg_$r.json" 2> "$O/bench_reg_$r.err" || exit 1
done
for f in "$O"/bench_*.json; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['p50_latency_ms'])" "$f"; done
