#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../../.."
out=gpurun_out/${1:-r6_tp8_var}
mkdir -p $out
export PYTHONUNBUFFERED=1
for v in eager_sync eager_pipelined decode_graphs all_graphs_sync all; do
  timeout -k 10 300 python scripts/archive/r6/tp8_variants.py $v > $out/$v.log 2>&1 || { echo "rc=$? on $v"; tail -5 $out/$v.log; exit 1; }
  grep '"variant"' $out/$v.log | cut -c1-600
done
