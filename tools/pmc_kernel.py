"""Per-kernel averages of rocprofv3 --pmc counter CSVs.

Usage: python tools/pmc_kernel.py DIR [kernel-substring] -- prints, per kernel
whose name contains the substring, the mean of every counter over its
dispatches, plus the derived clock (GRBM_GUI_ACTIVE / 8 XCDs / duration) and
MFMA busy fraction when those counters are present."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    acc = defaultdict(lambda: defaultdict(float))
    ndisp = defaultdict(set)
    dur = defaultdict(dict)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "")
                if pat not in name:
                    continue
                key = name[:90]
                did = row.get("Dispatch_Id")
                acc[key][row["Counter_Name"]] += float(row["Counter_Value"])
                ndisp[key].add(did)
                if "Start_Timestamp" in row and row.get("End_Timestamp"):
                    dur[key][did] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
    for k, cs in acc.items():
        n = len(ndisp[k])
        print(f"{k}  dispatches={n}")
        for c, v in sorted(cs.items()):
            print(f"   {c:28s} {v / n:.4g}")
        if dur[k]:
            ns = sum(dur[k].values()) / len(dur[k])
            print(f"   duration_ns                 {ns:.4g}")
            if "GRBM_GUI_ACTIVE" in cs:
                print(f"   clock_GHz                   {cs['GRBM_GUI_ACTIVE'] / n / 8 / ns:.3f}")
            if "SQ_VALU_MFMA_BUSY_CYCLES" in cs and "SQ_BUSY_CYCLES" in cs:
                print(f"   mfma_busy/busy              {cs['SQ_VALU_MFMA_BUSY_CYCLES'] / cs['SQ_BUSY_CYCLES']:.3f}")


if __name__ == "__main__":
    main()
