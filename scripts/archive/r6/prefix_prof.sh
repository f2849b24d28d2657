#!/bin/bash
# (runs against the tree with scripts/archive/decode_prefix_pass.patch applied; the pass is not shipped)
# Round 6: kernel times of the shared-prefix decode pass: rocprofv3 kernel trace of the
# 256 x 1,400 decode step with a 133-token shared head, prefix pass on and off
set -o pipefail
cd "$(dirname "$0")/../../.."
out=gpurun_out/${1:-r6_prefix_prof}
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD TMPDIR=/tmp
for pf in 1 0; do
  NGA_DECODE_PREFIX=$pf timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/pf$pf -o run -- python3 benchmarks/decode_step.py --batch 256 --ctx 1400 --steps 16 --shared-prefix 133 > $out/decode_pf$pf.json 2> $out/decode_pf$pf.err || { tail -20 $out/decode_pf$pf.err; exit 1; }
  f=$(find $out/pf$pf -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] || { echo "no kernel_stats.csv"; exit 1; }
  echo "== prefix=$pf $(tail -1 $out/decode_pf$pf.json)"
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    n = r["Name"]
    if "decode_attn" in n or "decode_prefix" in n or "skinny" in n.lower():
        print(f'{float(r["AverageNs"])/1e3:9.2f} us x {r["Calls"]:>6}  {n[:90]}')
PY
  rm -rf $out/pf$pf
done
