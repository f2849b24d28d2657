"""Join a rocprofv3 ``--kernel-trace --pmc`` run's counter and kernel-trace CSVs per dispatch
and summarise by (kernel, grid): mean duration, mean counter values and, when FETCH_SIZE /
WRITE_SIZE were collected, the HBM-side bandwidth those bytes imply over the dispatch's own
duration. Usage: pmc_summary.py <rocprofv3 output dir> [kernel-name substring ...]"""
import collections
import csv
import glob
import sys


def main():
    root = sys.argv[1]
    pats = sys.argv[2:]
    dur = {}
    for f in glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    per = collections.defaultdict(dict)
    meta = {}
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            if pats and not any(p in name for p in pats):
                continue
            d = r["Dispatch_Id"]
            per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            grid = r.get("Grid_Size", r.get("Grid_Size_X", "?"))
            meta[d] = (name.split("(")[0][:70], grid, r.get("LDS_Block_Size", r.get("Lds_Size", "?")),
                       r.get("VGPR_Count", r.get("Arch_VGPR_Count", "?")))
    groups = collections.defaultdict(list)
    for d, c in per.items():
        groups[meta[d]].append((dur.get(d), c))
    for (name, grid, lds, vgpr), rows in sorted(groups.items()):
        ds = [x for x, _ in rows if x is not None]
        mdur = sum(ds) / len(ds) if ds else float("nan")
        print(f"{name}  grid={grid} lds={lds} vgpr={vgpr}  dispatches={len(rows)}  mean_us={mdur:.1f}")
        keys = sorted({k for _, c in rows for k in c})
        for k in keys:
            v = [c[k] for _, c in rows if k in c]
            print(f"    {k:28s} {sum(v) / len(v):16.1f}")
        for k in ("FETCH_SIZE", "WRITE_SIZE"):
            pairs = [(x, c[k]) for x, c in rows if x and k in c]
            if pairs:   # KB per dispatch
                tb = sum(c * 1024 / x / 1e6 for x, c in pairs) / len(pairs)
                print(f"    {k} bandwidth (bytes / own duration) {tb:.2f} TB/s")
        cyc = [c for _, c in rows if "SQ_BUSY_CU_CYCLES" in c and "SQ_VALU_MFMA_BUSY_CYCLES" in c]
        if cyc:
            u = sum(c["SQ_VALU_MFMA_BUSY_CYCLES"] / max(1.0, c["SQ_BUSY_CU_CYCLES"]) for c in cyc) / len(cyc)
            print(f"    MFMA busy / CU busy cycles  {u:.3f}")


if __name__ == "__main__":
    main()
