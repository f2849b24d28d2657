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
        # SQ_VALU_MFMA_BUSY_CYCLES sums the issuing SIMD's cycles of every MFMA (16 per
        # 16x16x32 bf16, 32 per 32x32x16: 1,024 FLOP per counted cycle for both shapes), over
        # all SIMDs; SQ_BUSY_CU_CYCLES sums busy cycles over CUs (~256 x the dispatch's cycles).
        # A CU has 4 SIMDs, so utilisation = MFMA_BUSY / (4 x BUSY_CU), in [0, 1].
        cyc = [(x, c) for x, c in rows if "SQ_BUSY_CU_CYCLES" in c and "SQ_VALU_MFMA_BUSY_CYCLES" in c]
        if cyc:
            u = sum(c["SQ_VALU_MFMA_BUSY_CYCLES"] / max(1.0, 4.0 * c["SQ_BUSY_CU_CYCLES"]) for _, c in cyc) / len(cyc)
            print(f"    MFMA utilisation (MFMA busy / 4 SIMDs x CU busy)  {u:.3f}")
            fl = [1024.0 * c["SQ_VALU_MFMA_BUSY_CYCLES"] / (x * 1e-6) for x, c in cyc if x]
            if fl:
                print(f"    MFMA FLOP/s implied by the counter (1,024 FLOP per busy cycle)  "
                      f"{sum(fl) / len(fl) / 1e12:.1f} TFLOP/s")
        # HBM read bytes from the raw TCC->EA request counters by size (the FETCH_SIZE derived
        # formula of ROCm 7.2 is the gfx94x one, which prices gfx950's 128-B requests at 64 B)
        req = [(x, c) for x, c in rows if "TCC_EA0_RDREQ_sum" in c]
        if req:
            def rd_bytes(c):
                n = c["TCC_EA0_RDREQ_sum"]
                n32 = c.get("TCC_EA0_RDREQ_32B_sum", 0.0)
                n128 = c.get("TCC_EA0_RDREQ_128B_sum", None)
                n64 = c.get("TCC_EA0_RDREQ_64B_sum", None)
                if n128 is None:   # size split not collected: 32 B and 64 B requests assumed
                    return 32 * n32 + 64 * (n - n32)
                if n64 is None:
                    n64 = max(0.0, n - n32 - n128)
                return 32 * n32 + 64 * n64 + 128 * n128
            by = [rd_bytes(c) for _, c in req]
            print(f"    HBM read bytes (TCC_EA0_RDREQ by size)  {sum(by) / len(by) / 1e6:.1f} MB")
            bw = [rd_bytes(c) / (x * 1e-6) for x, c in req if x]
            if bw:
                print(f"    HBM read bandwidth (bytes / own duration)  {sum(bw) / len(bw) / 1e12:.2f} TB/s")


if __name__ == "__main__":
    main()
