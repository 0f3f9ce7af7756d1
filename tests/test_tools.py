"""CPU: the measurement tools the profiles/ records come from -- the PMC
summary (FETCH_SIZE x2 + WRITE_SIZE per dispatch, several kernels summed,
a grid filter) and the kernel-trace summary (busy time as the union of the
insert kernels' intervals) -- on small synthetic rocprofv3-style CSVs."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _write(path, header, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(header)
        w.writerows(rows)


def test_pmc_summary_sums_kernels(tmp_path):
    hdr = ["Dispatch_Id", "Kernel_Name", "Grid_Size", "Counter_Name", "Counter_Value"]
    _write(str(tmp_path / "f" / "run_counter_collection.csv"), hdr, [
        [1, "void mh::k_batch_search<x>", 64, "FETCH_SIZE", 100.0],
        [2, "void mh::k_batch_search<x>", 128, "FETCH_SIZE", 300.0],
        [3, "void mh::k_batch_commit<x>", 64, "FETCH_SIZE", 10.0],
        [4, "void mh::k_search_beam<x>", 4194304, "FETCH_SIZE", 7.0],
    ])
    _write(str(tmp_path / "w" / "run_counter_collection.csv"), hdr, [
        [1, "void mh::k_batch_search<x>", 64, "WRITE_SIZE", 1.0],
        [2, "void mh::k_batch_search<x>", 128, "WRITE_SIZE", 3.0],
        [3, "void mh::k_batch_commit<x>", 64, "WRITE_SIZE", 2.0],
    ])
    out = tmp_path / "o.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), str(tmp_path / "f"),
                    str(tmp_path / "w"), "k_batch_search+k_batch_commit<", str(out), "rev=t", "n=5"],
                   check=True, capture_output=True)
    r = json.load(open(out))
    # KB units: 2 x fetch + write, per dispatch summed
    assert r["per_kernel"]["k_batch_search"]["hbm_bytes_total"] == int((2 * 400 + 4) * 1024)
    assert r["per_kernel"]["k_batch_commit<"]["hbm_bytes_total"] == int((2 * 10 + 2) * 1024)
    assert r["hbm_bytes_total"] == int((2 * 410 + 6) * 1024)
    assert r["dispatches"] == 3 and r["rev"] == "t" and r["n"] == 5
    # one kernel, one grid size
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), str(tmp_path / "f"),
                    str(tmp_path / "w"), "k_batch_search@128", str(out)], check=True, capture_output=True)
    r = json.load(open(out))
    assert r["dispatches"] == 1 and r["hbm_bytes_per_launch"] == int((2 * 300 + 3) * 1024)


def test_trace_build_busy_union(tmp_path):
    hdr = ["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Grid_Size", "Workgroup_Size"]
    _write(str(tmp_path / "run_kernel_trace.csv"), hdr, [
        ["void mh::k_batch_search<x>(args)", 0, 1_000_000, 64 * 100, 64],        # 100 inserts, 1 ms
        ["void mh::k_batch_commit<x>(args)", 500_000, 1_500_000, 64 * 10, 64],   # overlaps 0.5 ms
        ["void mh::k_batch_search_mw<x>(args)", 2_000_000, 2_200_000, 256, 256],  # 1 insert
        ["void mh::k_search_beam<x>(args)", 3_000_000, 4_000_000, 64 * 8, 64],
    ])
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "trace_build.py"), str(tmp_path)],
                       check=True, capture_output=True, text=True)
    out = p.stdout
    assert "sum of durations 2.2 ms, busy (union) 1.7 ms, first start to last end 2.2 ms" in out
    assert "inserts<=      1 launches=   1" in out and "inserts<=    128 launches=   1" in out
