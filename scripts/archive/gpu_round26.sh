#!/usr/bin/env bash
# Concurrent prefill/decode attention in mixed steps: numerics, mixed-step micro-bench, bench.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="$R/gpurun_out/r26"
mkdir -p "$O"
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q -p no:cacheprovider \
    --timeout 200 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
timeout -k 10 300 python benchmarks/mixed_step.py --decode 256 --ctx 1330 --prefill 1170 > "$O/mixed.log" 2>&1 || { tail -20 "$O/mixed.log"; exit 1; }
grep '^{' "$O/mixed.log"
timeout -k 10 300 python benchmarks/mixed_step.py --decode 256 --ctx 1330 --prefill 600,570 > "$O/mixed2.log" 2>&1 || { tail -20 "$O/mixed2.log"; exit 1; }
grep '^{' "$O/mixed2.log"
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --out "$O/bench.json" > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log" | cut -c1-250
NGA_CONCURRENT_ATTN=0 timeout -k 10 600 python bench.py --steps 2 --warmup 1 --out "$O/bench_seq.json" > "$O/bench_seq.log" 2>&1 || { tail -20 "$O/bench_seq.log"; exit 1; }
tail -1 "$O/bench_seq.log" | cut -c1-250
