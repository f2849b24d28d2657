#!/bin/bash
# Round 5: the driver's configuration on the final tree, then a kernel table of a short headline run
set -o pipefail
cd "$(dirname "$0")/../.."
R=$PWD
out=gpurun_out/r5_final3
mkdir -p $out
timeout -k 10 700 python bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$out/bench.json'));print(d['value'], d['p50_latency_ms'], d['p50_ttft_ms'], d['prefix_cache'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$out/raw -o run -- python3 $R/bench.py --steps 3 --warmup 1 > $R/$out/prof.log 2>&1 || { tail -20 $R/$out/prof.log; exit 1; }
python3 $R/scripts/summarize_prof.py $R/$out/raw > $R/$out/kernels.txt 2>&1
rm -rf $R/$out/raw
head -12 $R/$out/kernels.txt
