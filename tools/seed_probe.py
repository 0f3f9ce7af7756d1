"""The bench index (bench.py's graph: 1M x 768 cosine, latent 12, M 16, M0 40, efC 400,
upper_efc 128, slack 1.15, batches of 20 %, build_expand 4) built from other data seeds:
recall@10 at ef 48 / 64 / 72 against the exact path on 4,096 queries, QPS at ef 64 on
65,536-query batches.  Usage: python tools/seed_probe.py [seed ...]"""
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import hnsw_amd as H  # noqa: E402
from bench import Searcher, gen_vectors, recall_at_k  # noqa: E402

dev = torch.device("cuda")
n, d, B = 1_000_000, 768, 65536
for seed in [int(a) for a in sys.argv[1:]] or [1234]:
    X = gen_vectors(n, d, seed, 12, 1000, dev, "cosine")
    Q = gen_vectors(B, d, seed + 7777, 12, 1000, dev, "cosine")
    g = H.Graph(M=16, Ml=0.25, EfSearch=64, Distance=H.CosineDistance, Rng=seed, build_mode=H.BUILD_BATCH, m0=40,
                ef_construction=400, heuristic=2, keep_pruned=1, prune_alpha_pct=115, build_expand=4,
                batch_ratio_pct=20, upper_efc=128)
    g.reserve(n, d)
    g.add_device(np.arange(n), X.data_ptr(), n, d)
    del X
    tk, _, tn = (x.clone() for x in Searcher(g, 4096, 10, d, dev).run(Q[:4096], H.MODE_EXACT, 0))
    S = Searcher(g, B, 10, d, dev)
    out = []
    for ef in (48, 64, 72):
        kk, _, nn = (x.clone() for x in S.run(Q, H.MODE_BEAM, ef))
        out.append(f"ef {ef}: {recall_at_k(kk[:4096], nn[:4096], tk, tn, 10):.4f}")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        S.run(Q, H.MODE_BEAM, 64)
    torch.cuda.synchronize()
    print(f"seed {seed}: recall@10 " + ", ".join(out) + f"; {B * 3 / (time.perf_counter() - t0) / 1e6:.3f} M queries/s at ef 64",
          flush=True)
    g.close()
    del Q
    torch.cuda.empty_cache()
