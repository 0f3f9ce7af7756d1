"""Summarise rocprofv3 --pmc counter CSVs into per-launch HBM traffic for one
kernel (MI355X_MICROARCH.md 'HBM': FETCH_SIZE reports 1/2 of the bytes of a
wide coalesced streaming read on gfx950 -> doubled; WRITE_SIZE exact for
16-B/lane stores).  Usage:
  python tools/pmc_summary.py FETCH_DIR WRITE_DIR KERNEL_SUBSTR[@GRID] OUT.json key=value...
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
    fdir, wdir, kernel, out = sys.argv[1:5]
    extra = dict(kv.split("=", 1) for kv in sys.argv[5:])
    f = per_dispatch(fdir, "FETCH_SIZE", kernel)
    w = per_dispatch(wdir, "WRITE_SIZE", kernel)
    if not f:
        raise SystemExit("no FETCH_SIZE rows for " + kernel)
    fk = sum(f) / len(f)
    wk = sum(w) / len(w) if w else 0.0
    res = {
        "kernel": kernel,
        "dispatches": len(f),
        "fetch_size_kb_raw": fk,
        "write_size_kb": wk,
        "hbm_bytes_per_launch": int(2 * fk * 1024 + wk * 1024),
        "hbm_bytes_total": int((2 * fk * 1024 + wk * 1024) * len(f)),
        "correction": "FETCH_SIZE x2 (gfx950 wide-load half count), WRITE_SIZE x1; KB units",
    }
    for k, v in extra.items():
        try:
            res[k] = int(v)
        except ValueError:
            res[k] = v
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
