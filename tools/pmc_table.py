"""Per-kernel mean of every PMC counter in the rocprofv3 counter CSVs under a
directory (one value per dispatch summed over its rows, then averaged).
Usage: python tools/pmc_table.py DIR [kernel-substring ...]"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
subs = sys.argv[2:]
per = collections.defaultdict(float)
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        per[(r["Kernel_Name"], f, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for (k, _, _, c), v in per.items():
    if not subs or any(s in k for s in subs):
        agg[k][c].append(v)
for k, cs in agg.items():
    print(k[:70])
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v) / len(v):16.0f}  (n={len(v)})")
