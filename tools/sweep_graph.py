"""GPU sweep: graph build settings -> recall@10 and batched-search QPS on the
bench workload (1M x 768 cosine).  python tools/sweep_graph.py [n]"""
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import hnsw_amd as H  # noqa: E402
from bench import Searcher, gen_vectors, recall_at_k  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
which = sys.argv[2] if len(sys.argv) > 2 else "base"
dev = torch.device("cuda")
X = gen_vectors(n, 768, 1234, 12, 1000, dev, "cosine")
Q = gen_vectors(16384, 768, 1234 + 7777, 12, 1000, dev, "cosine")
configs = [
    dict(M=16, m0=32, ef_construction=400, heuristic=2, keep_pruned=1),
    dict(M=16, m0=40, ef_construction=400, heuristic=2, keep_pruned=1),
    dict(M=16, m0=40, ef_construction=400, heuristic=2),
    dict(M=16, m0=48, ef_construction=400, heuristic=2, keep_pruned=1),
    dict(M=16, m0=32, ef_construction=512, heuristic=2, keep_pruned=1),
    dict(M=12, m0=32, ef_construction=400, heuristic=2, keep_pruned=1),
]
if which == "alpha":  # heuristic slack (prune_alpha_pct) on the bench graph
    configs = [dict(M=16, m0=48, ef_construction=400, heuristic=2, keep_pruned=1, prune_alpha_pct=a)
               for a in (100, 90, 115, 130)]
    configs.append(dict(M=16, m0=48, ef_construction=400, heuristic=2, keep_pruned=0, prune_alpha_pct=120))
EFS = (64, 72, 80, 88, 96)
if which == "alpha2":  # finer: the ef at which each slack first reaches recall 0.99
    configs = [dict(M=16, m0=48, ef_construction=400, heuristic=2, keep_pruned=1, prune_alpha_pct=a)
               for a in (105, 110, 115, 120)]
    EFS = (48, 56, 64, 72)
if which == "alpha3":  # slack x layer-0 degree
    configs = [dict(M=16, m0=m0, ef_construction=400, heuristic=2, keep_pruned=1, prune_alpha_pct=a)
               for (a, m0) in ((110, 40), (115, 40), (120, 40), (110, 44), (115, 44), (120, 32))]
    EFS = (56, 64, 72)
for cfg in configs:
    cfg = dict(cfg)
    M = cfg.pop("M")
    g = H.Graph(M=M, Ml=0.25, EfSearch=64, Distance=H.CosineDistance, Rng=1234, build_mode=H.BUILD_BATCH, **cfg)
    g.reserve(n, 768)
    torch.cuda.synchronize()
    t0 = time.time()
    g.add_device(np.arange(n), X.data_ptr(), n, 768)
    torch.cuda.synchronize()
    bt = time.time() - t0
    G = Searcher(g, 4096, 10, 768, dev)
    tk, td, tn = (x.clone() for x in G.run(Q[:4096], H.MODE_EXACT, 0))
    S = Searcher(g, 16384, 10, 768, dev)
    for ef in EFS:
        S.run(Q, H.MODE_BEAM, ef)
        torch.cuda.synchronize()
        t0 = time.time()
        for _ in range(5):
            k_, d_, n_ = S.run(Q, H.MODE_BEAM, ef)
        torch.cuda.synchronize()
        dt = (time.time() - t0) / 5
        r = recall_at_k(k_[:4096], n_[:4096], tk, tn, 10)
        print(f"M={M} {cfg} build={bt:.1f}s ef={ef} recall@10={r:.4f} qps={16384 / dt / 1e6:.3f}M", flush=True)
    g.close()
