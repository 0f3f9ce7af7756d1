"""BASELINE configs[2] (1M x 768 L2 batched insert, M 16, M0 48, efC 64, batches of 20 %,
build_expand 4) with other batch schedules / options: inserts/s, the insert kernels'
time and recall@10 at ef 64 on 4,096 queries.
Usage: python tools/config2_sched_probe.py [opt=v:opt=v ...]   ('-' = the bench's settings)"""
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import hnsw_amd as H  # noqa: E402
from bench import Searcher, gen_vectors, recall_at_k  # noqa: E402

dev = torch.device("cuda")
n, d = 1_000_000, 768
X = gen_vectors(n, d, 77, 12, 1000, dev, "euclidean")
Q = gen_vectors(4096, d, 78, 12, 1000, dev, "euclidean")
for arg in sys.argv[1:] or ["-"]:
    kw = dict(m0=48, ef_construction=64, heuristic=2, batch_ratio_pct=20, build_expand=4, time_build=1)
    if arg != "-":
        kw.update({k: int(v) for k, v in (kv.split("=") for kv in arg.split(":"))})
    g = H.Graph(M=16, Ml=0.25, EfSearch=64, Distance=H.EuclideanDistance, Rng=5, build_mode=H.BUILD_BATCH, **kw)
    g.reserve(n, d)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g.add_device(np.arange(n), X.data_ptr(), n, d)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st = g.stats()
    tk, _, tn = (x.clone() for x in Searcher(g, 4096, 10, d, dev).run(Q, H.MODE_EXACT, 0))
    k_, _, n_ = Searcher(g, 4096, 10, d, dev).run(Q, H.MODE_BEAM, 64)
    print(f"{arg}: {n / dt:.0f} inserts/s ({dt:.3f} s), insert kernels {st['build_search_us'] / 1e6:.3f} s, "
          f"recall@10 ef 64 {recall_at_k(k_, n_, tk, tn, 10):.4f}", flush=True)
    g.close()
