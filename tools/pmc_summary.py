"""Summarise rocprofv3 --pmc counter CSVs into per-launch HBM traffic for one
kernel (MI355X_MICROARCH.md 'HBM': FETCH_SIZE reports 1/2 of the bytes of a
wide coalesced streaming read on gfx950 -> doubled; WRITE_SIZE exact for
16-B/lane stores).  Usage:
  python tools/pmc_summary.py FETCH_DIR WRITE_DIR KERNEL_SUBSTR[@GRID][+KERNEL2...] OUT.json key=value...
('+' sums the HBM bytes of several kernels, e.g. the three insert kernels)
(@GRID keeps only the dispatches of that grid size, e.g. the headline batch's
launches of a kernel the same run also launches on smaller batches)
"""
import csv
import glob
import json
import os
import sys


def per_dispatch(d, counter, kernel):
    grid = None
    if "@" in kernel:
        kernel, grid = kernel.split("@")
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name") or r.get("Kernel-Name") or ""
            cname = r.get("Counter_Name") or r.get("Counter-Name") or ""
            if kernel in name and cname == counter and (grid is None or r.get("Grid_Size") == grid):
                did = r.get("Dispatch_Id") or r.get("Dispatch-Id") or str(len(vals))
                vals[did] = vals.get(did, 0.0) + float(r.get("Counter_Value") or r.get("Counter-Value") or 0)
    return list(vals.values())


def main():
    fdir, wdir, kernels, out = sys.argv[1:5]
    extra = dict(kv.split("=", 1) for kv in sys.argv[5:])
    res = {"kernel": kernels, "dispatches": 0, "fetch_size_kb_raw": 0.0, "write_size_kb": 0.0,
           "hbm_bytes_total": 0, "per_kernel": {}}
    for kernel in kernels.split("+"):
        f = per_dispatch(fdir, "FETCH_SIZE", kernel)
        w = per_dispatch(wdir, "WRITE_SIZE", kernel)
        if not f:
            raise SystemExit("no FETCH_SIZE rows for " + kernel)
        tot = int(2 * sum(f) * 1024 + sum(w) * 1024)
        res["per_kernel"][kernel] = {"dispatches": len(f), "hbm_bytes_total": tot}
        res["dispatches"] += len(f)
        res["fetch_size_kb_raw"] += sum(f) / len(f)
        res["write_size_kb"] += sum(w) / len(w) if w else 0.0
        res["hbm_bytes_total"] += tot
    # per launch of the (single) kernel; for a '+' list, the sum of each kernel's mean
    res["hbm_bytes_per_launch"] = int(2 * res["fetch_size_kb_raw"] * 1024 + res["write_size_kb"] * 1024)
    res["correction"] = "FETCH_SIZE x2 (gfx950 wide-load half count), WRITE_SIZE x1; KB units"
    for k, v in extra.items():
        try:
            res[k] = int(v)
        except ValueError:
            res[k] = v
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
