"""Headline-search knob probe on the bench graph (1M x 768 cosine, bench.py
defaults): QPS / recall / distance evals / visited resets per setting.
Usage: python tools/search_probe.py [name=value ...]  (default: the knob list below)
Env: PROBE_BATCH (16384), PROBE_LATENT (12: the bench data), PROBE_EFS ("56,64")."""
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import hnsw_amd as H  # noqa: E402
from bench import Searcher, gen_vectors, recall_at_k  # noqa: E402

dev = torch.device("cuda")
n, d, B = 1_000_000, 768, int(os.environ.get("PROBE_BATCH", 16384))
lat = int(os.environ.get("PROBE_LATENT", 12))
efs = [int(x) for x in os.environ.get("PROBE_EFS", "56,64").split(",")]
X = gen_vectors(n, d, 1234, lat, 1000, dev, "cosine")
Q = gen_vectors(B, d, 1234 + 7777, lat, 1000, dev, "cosine")
g = H.Graph(M=16, Ml=0.25, EfSearch=64, Distance=H.CosineDistance, Rng=1234, build_mode=H.BUILD_BATCH, m0=40,
            ef_construction=400, heuristic=2, keep_pruned=1, prune_alpha_pct=115)
g.reserve(n, d)
g.add_device(np.arange(n), X.data_ptr(), n, d)
del X
G = Searcher(g, 4096, 10, d, dev)
tk, td, tn = (x.clone() for x in G.run(Q[:4096], H.MODE_EXACT, 0))
S = Searcher(g, B, 10, d, dev)
knobs = [("vis_log2", 12), ("upper_ef", 1), ("upper_ef", 4), ("upper_ef", 16)]
if sys.argv[1:]:
    knobs = [(kv.split("=")[0], int(kv.split("=")[1])) for kv in sys.argv[1:]]
for name, val in knobs:
    g.set_option(name, val)
    vl = f"{name}={val}"
    for ef in efs:
        S.run(Q, H.MODE_BEAM, ef)
        g.reset_stats()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            k_, _, n_ = S.run(Q, H.MODE_BEAM, ef)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 5
        st = g.stats()
        r = recall_at_k(k_[:4096], n_[:4096], tk, tn, 10)
        print(f"{vl} ef={ef} qps={B / dt / 1e6:.3f}M recall={r:.4f} E={st['search_dist_evals'] / 5 / B:.1f} "
              f"S={st['search_screened'] / 5 / B:.1f} F={st['search_f32_evals'] / 5 / B:.1f} "
              f"resets/q={st['visited_resets'] / 5 / B:.3f} kernel_ms={g.last_kernel_ms():.3f}", flush=True)
