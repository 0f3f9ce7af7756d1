"""Single-query latency (SURVEY 8(d) C2 batch points) on the bench index (bench.py's graph:
1M x 768 cosine, efC 400, upper_efc 128) at ef 64 for each layer-0 expansion width
(search_expand 1 runs the 4-wave small-batch kernel below 512 queries; 2 and 4 the
one-wave kernel): ms per batch of B queries, recall@10 on the first 1,024 queries.
Usage: python tools/latency_probe.py"""
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
X = gen_vectors(n, d, 1234, 12, 1000, dev, "cosine")
Q = gen_vectors(10000, d, 1234 + 7777, 12, 1000, dev, "cosine")
g = H.Graph(M=16, Ml=0.25, EfSearch=64, Distance=H.CosineDistance, Rng=1234, build_mode=H.BUILD_BATCH, m0=40,
            ef_construction=400, heuristic=2, keep_pruned=1, prune_alpha_pct=115, build_expand=4, batch_ratio_pct=20,
            upper_efc=128)
g.reserve(n, d)
g.add_device(np.arange(n), X.data_ptr(), n, d)
del X
tk, _, tn = (x.clone() for x in Searcher(g, 1024, 10, d, dev).run(Q[:1024], H.MODE_EXACT, 0))
for xw in (1, 2, 4):
    g.set_option("search_expand", xw)
    kk, _, nn = (x.clone() for x in Searcher(g, 1024, 10, d, dev).run(Q[:1024], H.MODE_BEAM, 64))
    r = recall_at_k(kk, nn, tk, tn, 10)
    out = []
    for B in (1, 16, 256, 1024, 10000):
        S = Searcher(g, B, 10, d, dev)
        Qb = Q[:B].contiguous()
        S.run(Qb, H.MODE_BEAM, 64)
        reps = max(5, min(500, 200_000 // B))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            S.run(Qb, H.MODE_BEAM, 64)
        torch.cuda.synchronize()
        out.append(f"B={B}: {(time.perf_counter() - t0) / reps * 1e3:.3f} ms")
    print(f"search_expand {xw}: recall@10 (1,024 queries) {r:.4f}; " + ", ".join(out), flush=True)
g.close()
