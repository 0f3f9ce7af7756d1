"""The distance sweep (mhnsw_sweep_device, bench.py's sweep leg) alone: one
query against 1M x 768 rows, cosine and L2, HIP events over 20 sweeps; for
comparing tools/Makefile.beam builds of search.hip (MH_SWEEP_* flags).
Usage: python tools/sweep_probe.py"""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import hnsw_amd as H  # noqa: E402

n, d, reps = 1_000_000, 768, 20
dev = torch.device("cuda")
X = torch.randn(n, d, device=dev)
q = torch.randn(d, device=dev)
out = torch.empty(n, device=dev)
s = torch.cuda.current_stream()
for metric, name in ((H.CosineDistance.metric, "cosine"), (H.EuclideanDistance.metric, "l2")):
    H.sweep_device(metric, q.data_ptr(), X.data_ptr(), n, d, out.data_ptr(), s.cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        H.sweep_device(metric, q.data_ptr(), X.data_ptr(), n, d, out.data_ptr(), s.cuda_stream)
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(f"{name}: {ms:.4f} ms per sweep = {n * d * 4 / ms / 1e6:.0f} GB/s = {n * d * 4 / ms / 1e6 / 8000:.3f} of 8 TB/s",
          flush=True)
