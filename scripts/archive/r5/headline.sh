#!/bin/bash
# Round 5: headline at the driver configuration (20 steps, 5 warm-up) with and without the
# prefix cache, the decode step at 256 x 1,400, and a kernel table of the headline
set -o pipefail
cd "$(dirname "$0")/../.."
R=$PWD
out=gpurun_out/${1:-r5_headline}
mkdir -p $out
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench.json'));print('default', d['value'],d['p50_latency_ms'],d['p50_ttft_ms'],d['prefix_cache'],d.get('gpu_step_timing'))"
timeout -k 10 500 python bench.py --steps 20 --warmup 5 --no-prefix-cache > $out/bench_nopc.json 2> $out/bench_nopc.err || { tail -20 $out/bench_nopc.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench_nopc.json'));print('no-prefix-cache', d['value'],d['p50_latency_ms'],d['p50_ttft_ms'],d['prefix_cache'])"
timeout -k 10 300 python benchmarks/decode_step.py --batch 256 --ctx 1400 --steps 16 > $out/decode256.json 2> $out/decode256.err || { tail -20 $out/decode256.err; exit 1; }
tail -2 $out/decode256.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$out/raw -o run -- python3 $R/bench.py --steps 6 --warmup 3 > $R/$out/prof.log 2>&1 || { tail -20 $R/$out/prof.log; exit 1; }
python3 $R/scripts/summarize_prof.py $R/$out/raw > $R/$out/kernels.txt 2>&1
rm -rf $R/$out/raw
head -30 $R/$out/kernels.txt
