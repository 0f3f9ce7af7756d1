"""Summarise a rocprofv3 --kernel-trace CSV of a bench run: per kernel (and,
for k_search_beam, per grid size) dispatches / mean / total ms, and for the
batched insert's kernels (k_batch_*) the sum of their durations against the
time the GPU was busy with at least one of them (the union of their
intervals: below the sum only when kernels run concurrently),
plus k_batch_search* by launch width.
Usage: python tools/trace_build.py TRACE_DIR_OR_CSV"""
import csv
import glob
import os
import sys
from collections import defaultdict


def rows(path):
    files = [path] if path.endswith(".csv") else glob.glob(os.path.join(path, "**", "*kernel_trace*.csv"),
                                                           recursive=True)
    for f in files:
        for r in csv.DictReader(open(f)):
            yield r


def main():
    per = defaultdict(list)
    build = []
    width = defaultdict(lambda: [0, 0.0, 0])
    for r in rows(sys.argv[1]):
        name = r.get("Kernel_Name") or ""
        t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        grid = int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)
        wg = int(r.get("Workgroup_Size") or r.get("Workgroup_Size_X") or 64)
        short = name.split("(")[0]
        key = short + (f" grid={grid}" if short.startswith("k_search_beam<") else "")
        per[key].append((t1 - t0) / 1e6)
        if "k_batch_" in short:
            build.append((t0, t1))
        if "k_batch_search" in short:
            inserts = grid // wg
            b = 1
            while b < inserts:
                b *= 2
            width[b][0] += 1
            width[b][1] += (t1 - t0) / 1e6
            width[b][2] += inserts
    for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        print(f"{k[:90]:90s} n={len(v):5d} mean_ms={sum(v) / len(v):9.4f} total_ms={sum(v):10.2f}")
    if build:
        build.sort()
        busy, cur0, cur1 = 0, build[0][0], build[0][1]
        for a, b in build[1:]:
            if a > cur1:
                busy += cur1 - cur0
                cur0, cur1 = a, b
            else:
                cur1 = max(cur1, b)
        busy += cur1 - cur0
        tot = sum(b - a for a, b in build)
        span = max(b for _, b in build) - build[0][0]
        print(f"# insert kernels: sum of durations {tot / 1e6:.1f} ms, busy (union) {busy / 1e6:.1f} ms, "
              f"first start to last end {span / 1e6:.1f} ms")
        print("# k_batch_search* by launch width (inserts searched in that launch and layer)")
        for b in sorted(width):
            n, ms, ins = width[b]
            print(f"inserts<={b:7d} launches={n:4d} ms={ms:8.1f} inserts={ins:8d} us/insert={ms * 1e3 / max(ins, 1):8.3f}")


if __name__ == "__main__":
    main()
