#!/bin/bash
# Kernel-busy time over bench.py's timed window: rocprofv3 kernel trace of 8 timed steps, cut at
# the marker kernels bench.py launches around its timed region (scripts/summarize_prof.py).
# Usage: gpu_busy.sh [out-name]
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
out=gpurun_out/${1:-busy}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$out/raw -o run -- python3 $R/bench.py --steps 8 --warmup 2 --out $R/$out/bench_traced.json > $R/$out/prof.log 2>&1 || { tail -20 $R/$out/prof.log; exit 1; }
python3 $R/scripts/summarize_prof.py $R/$out/raw > $R/$out/kernels.txt 2>&1
rm -rf $R/$out/raw
grep -A 20 "gpu busy" $R/$out/kernels.txt | head -24
