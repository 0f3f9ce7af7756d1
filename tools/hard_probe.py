"""Harder-data search probe for counter passes: the bench's latent-32 set
(1M x 768 cosine, M 32, M0 63, efConstruction 512), then `reps` searches of
16,384 queries at each ef given (k_search_beam R = 1 at ef 64, R = 8 at 512:
separate kernels in a trace), for each vis_compact value given (1: the compact
16-bit visited set, 0: the 32-bit one).
Usage: python tools/hard_probe.py [efs=64,512] [reps=2] [n] [compact=1]"""
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import hnsw_amd as H  # noqa: E402
from bench import Searcher, gen_vectors  # noqa: E402

efs = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "64,512").replace("+", ",").split(",")]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
n = int(sys.argv[3]) if len(sys.argv) > 3 else 1_000_000
cvals = [int(x) for x in (sys.argv[4] if len(sys.argv) > 4 else "1").split("+")]
d, batch = 768, 16384
dev = torch.device("cuda")
X = gen_vectors(n, d, 4321, 32, 1000, dev, "cosine")
Q = gen_vectors(batch, d, 4321 + 7777, 32, 1000, dev, "cosine")
g = H.Graph(M=32, Ml=0.25, EfSearch=64, Distance=H.CosineDistance, Rng=5, build_mode=H.BUILD_BATCH, m0=63,
            ef_construction=512, heuristic=2, keep_pruned=1, prune_alpha_pct=115, build_expand=2, screen=1)
g.reserve(n, d)
g.add_device(np.arange(n), X.data_ptr(), n, d)
del X
S = Searcher(g, batch, 10, d, dev)
for ef in efs:
    for c in cvals:
        g.set_option("vis_compact", c)
        S.run(Q, H.MODE_BEAM, ef)
        torch.cuda.synchronize()
        g.reset_stats()
        t0 = time.perf_counter()
        for _ in range(reps):
            S.run(Q, H.MODE_BEAM, ef)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        st = g.stats()
        print(f"ef={ef} vis_compact={c} ms={dt * 1e3:.2f} E/q={st['search_dist_evals'] / reps / batch:.1f} "
              f"F/q={st['search_f32_evals'] / reps / batch:.1f} X/q={st['search_expansions'] / reps / batch:.1f} "
              f"resets/q={st['visited_resets'] / reps / batch:.2f}", flush=True)
g.close()
