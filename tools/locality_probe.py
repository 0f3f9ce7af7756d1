"""Probe: does processing spatially-close queries together (per XCD) cut the
beyond-L2 traffic of k_search_beam?  Variants: original order; sorted by
nearest of 1000 anchor rows; sorted + XCD-contiguous block mapping
(blocks b and b+8 share an XCD)."""
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import hnsw_amd as H  # noqa: E402
from bench import Searcher, gen_vectors  # noqa: E402

dev = torch.device("cuda")
n, B = 1_000_000, 16384
X = gen_vectors(n, 768, 1234, 12, 1000, dev, "cosine")
Q = gen_vectors(B, 768, 9011, 12, 1000, dev, "cosine")
g = H.Graph(M=16, Ml=0.25, EfSearch=64, Distance=H.CosineDistance, Rng=1234, build_mode=H.BUILD_BATCH, m0=48,
            ef_construction=200, heuristic=2)
g.reserve(n, 768)
g.add_device(np.arange(n), X.data_ptr(), n, 768)
anchors = X[torch.randperm(n, device=dev)[:1000]]
key = (Q @ anchors.T).argmax(dim=1)
order = torch.argsort(key, stable=True)
Qs = Q[order].contiguous()
nx = 8
per = (B + nx - 1) // nx
b = torch.arange(B, device=dev)
p = (b % nx) * per + b // nx
p = torch.clamp(p, max=B - 1)
Qx = Qs[p].contiguous()
S = Searcher(g, B, 10, 768, dev)
for name, q in (("original", Q), ("anchor-sorted", Qs), ("sorted+xcd", Qx), ("original", Q)):
    S.run(q, H.MODE_BEAM, 64)
    torch.cuda.synchronize()
    g.reset_stats()
    t0 = time.time()
    ms = []
    for _ in range(5):
        S.run(q, H.MODE_BEAM, 64)
        ms.append(g.last_kernel_ms())
    torch.cuda.synchronize()
    dt = (time.time() - t0) / 5
    st = g.stats()
    print(f"{name:14s} qps={B / dt / 1e6:.3f}M kernel_ms={np.mean(ms):.3f} evals/q={st['search_dist_evals'] / 5 / B:.1f}",
          flush=True)
