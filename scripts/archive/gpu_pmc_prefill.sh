#!/usr/bin/env bash
# PMC counters for the prefill attention kernel (counters only; no trace domains).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/pmc"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d "$O/raw1" -o run -- python3 "$R/benchmarks/kernel_bench.py" --only prefill --iters 3 > "$O/run1.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM --output-format csv -d "$O/raw2" -o run -- python3 "$R/benchmarks/kernel_bench.py" --only prefill --iters 3 > "$O/run2.log" 2>&1; echo "run2 $?"
python3 - "$O" <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for f in glob.glob(f"{o}/raw*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")[:60]
        if "prefill" not in k:
            continue
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[(k, r["Counter_Name"])] += 1
with open(f"{o}/summary.txt", "w") as fh:
    for k, d in agg.items():
        fh.write(k + "\n")
        for c, v in sorted(d.items()):
            fh.write(f"  {c:24s} {v:16.0f}  (dispatches {cnt[(k, c)]})\n")
print(open(f"{o}/summary.txt").read())
PY
rm -rf "$O"/raw1 "$O"/raw2
