"""The harder-data graph (bench.config_harder's build: latent 32, 1M x 768 cosine,
M 32, M0 63, efC 512, build_expand 4, upper_efc 256) searched at ef 416-512 with
search_expand 4 and each upper-layer descent width given (option upper_ef): recall@10
against the exact path on 4,096 queries, QPS on 16,384-query batches.
Usage: python tools/harder_search_probe.py [upper_ef ...]"""
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import hnsw_amd as H  # noqa: E402
from bench import Searcher, gen_vectors, recall_at_k  # noqa: E402

dev = torch.device("cuda")
n, d, B = 1_000_000, 768, 16384
X = gen_vectors(n, d, 4321, 32, 1000, dev, "cosine")
Q = gen_vectors(B, d, 4321 + 7777, 32, 1000, dev, "cosine")
g = H.Graph(M=32, Ml=0.25, EfSearch=64, Distance=H.CosineDistance, Rng=5, build_mode=H.BUILD_BATCH, m0=63,
            ef_construction=512, heuristic=2, keep_pruned=1, prune_alpha_pct=115, build_expand=4, upper_efc=256,
            screen=1, batch_ratio_pct=20)
g.reserve(n, d)
g.add_device(np.arange(n), X.data_ptr(), n, d)
del X
tk, _, tn = (x.clone() for x in Searcher(g, 4096, 10, d, dev).run(Q[:4096], H.MODE_EXACT, 0))
S = Searcher(g, B, 10, d, dev)
g.set_option("search_expand", 4)
for ue in [int(a) for a in sys.argv[1:]] or [1]:
    g.set_option("upper_ef", ue)
    for ef in (416, 448, 480, 512):
        kk, _, nn = (x.clone() for x in S.run(Q, H.MODE_BEAM, ef))
        r = recall_at_k(kk[:4096], nn[:4096], tk, tn, 10)
        g.reset_stats()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            S.run(Q, H.MODE_BEAM, ef)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 3
        st = g.stats()
        print(f"upper_ef={ue} ef={ef}: recall {r:.4f}, {B / dt:.0f} queries/s, "
              f"{st['search_expansions'] / 3 / B:.1f} expansions/query", flush=True)
g.close()
