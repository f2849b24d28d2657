#!/bin/bash
# Interleaved A/B on one box: old tree (pageable embed-input copies) vs new (pinned).
set -o pipefail
O=gpurun_out/r3_ab_submit; mkdir -p $O
R=$(pwd)
for i in 1 2; do
  (cd $R/ab_old && timeout -k 10 400 python bench.py --steps 12 --warmup 3 > $R/$O/old_$i.json 2> $R/$O/old_$i.err) || exit 1
  python -c "import json;d=json.load(open('$O/old_$i.json'));print('old',d['value'],d['host_s'],d['host_work_ms']['submit'])"
  timeout -k 10 400 python bench.py --steps 12 --warmup 3 > $O/new_$i.json 2> $O/new_$i.err || exit 1
  python -c "import json;d=json.load(open('$O/new_$i.json'));print('new',d['value'],d['host_s'],d['host_work_ms']['submit'],d['submit_host_ms'])"
done
