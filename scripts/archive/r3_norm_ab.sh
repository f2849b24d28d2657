#!/bin/bash
# RMSNorm default back to the row-per-block form: norm tests (both forms), then the headline.
set -o pipefail
O=gpurun_out/r3_norm_ab; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "rmsnorm or layernorm" -x -v --timeout 120 --timeout-method thread > $O/test_norm.log 2>&1 || { tail -30 $O/test_norm.log; exit 1; }
tail -2 $O/test_norm.log
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['p50_latency_ms'],d['p50_ttft_ms'],d['host_s'])"
