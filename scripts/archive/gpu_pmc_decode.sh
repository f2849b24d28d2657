#!/usr/bin/env bash
# PMC counters for decode attention and the vector-search scoring kernel: HBM bytes fetched /
# written per dispatch (FETCH_SIZE / WRITE_SIZE, each in its own pass) with the kernel trace for
# durations, and SQ instruction mix. Counters only: no trace domains besides --kernel-trace.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/pmc_decode"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d "$O/$name" -o run -- \
      python3 "$R/benchmarks/kernel_bench.py" --only decode --iters 5 > "$O/$name.log" 2>&1
  echo "$name exit $?"
}
run fetch FETCH_SIZE || exit 1
run write WRITE_SIZE || exit 1
run sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_INSTS_LDS || exit 1
python3 - "$O" <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
durs = collections.defaultdict(list)
for f in glob.glob(f"{o}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")[:48]
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for f in glob.glob(f"{o}/fetch/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")[:48]
        durs[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
with open(f"{o}/summary.txt", "w") as fh:
    for k, d in vals.items():
        if "decode_attn" not in k:
            continue
        fh.write(k + "\n")
        for c, v in sorted(d.items()):
            fh.write(f"  {c:22s} mean/dispatch {sum(v) / len(v):16.1f}  (dispatches {len(v)})\n")
        if durs.get(k) and d.get("FETCH_SIZE"):
            # FETCH_SIZE is in KB; dispatches of all batch sizes mixed: report the largest
            fs = max(d["FETCH_SIZE"]) * 1024
            fh.write(f"  largest dispatch fetched {fs / 1e9:.3f} GB; longest dispatch {max(durs[k]):.1f} us;"
                     f" {fs / max(durs[k]) / 1e6:.2f} TB/s\n")
print(open(f"{o}/summary.txt").read())
PY
rm -rf "$O"/fetch "$O"/write "$O"/sq
