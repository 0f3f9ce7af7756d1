"""Batched insert of the bench index (1M x 768 cosine, bench.py's graph: M 16, M0 40,
efConstruction 400, slack 1.15, keep-pruned, batches of 20 %, build_expand 4) with a
narrower candidate list in the layers above 0 (option upper_efc): build time, the
insert kernels' time, and recall@10 / QPS of the built graph at ef 48 / 64 on 65,536
queries (recall against the exact path on 4,096 of them).
Usage: python tools/upper_efc_probe.py [upper_efc ...]   (0 = efConstruction everywhere)
       an argument may also be a colon-separated option list: upper_efc=128:batch_max=131072"""
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
X = gen_vectors(n, d, 1234, 12, 1000, dev, "cosine")
Q = gen_vectors(B, d, 1234 + 7777, 12, 1000, dev, "cosine")
for arg in sys.argv[1:] or ["0"]:
    opts = dict(kv.split("=") for kv in arg.split(":")) if "=" in arg else {"upper_efc": arg}
    kw = dict(build_expand=4, batch_ratio_pct=20, upper_efc=0)
    kw.update({k: int(v) for k, v in opts.items()})
    ue = arg
    g = H.Graph(M=16, Ml=0.25, EfSearch=64, Distance=H.CosineDistance, Rng=1234, build_mode=H.BUILD_BATCH, m0=40,
                ef_construction=400, heuristic=2, keep_pruned=1, prune_alpha_pct=115, time_build=1, **kw)
    g.reserve(n, d)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g.add_device(np.arange(n), X.data_ptr(), n, d)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st = g.stats()
    tk, _, tn = (x.clone() for x in Searcher(g, 4096, 10, d, dev).run(Q[:4096], H.MODE_EXACT, 0))
    S = Searcher(g, B, 10, d, dev)
    out = []
    for ef in (48, 64):
        kk, _, nn = (x.clone() for x in S.run(Q, H.MODE_BEAM, ef))
        r = recall_at_k(kk[:4096], nn[:4096], tk, tn, 10)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(3):
            S.run(Q, H.MODE_BEAM, ef)
        torch.cuda.synchronize()
        out.append(f"ef {ef}: recall {r:.4f} {B * 3 / (time.perf_counter() - t1) / 1e6:.3f} M q/s")
    print(f"upper_efc={ue}: {n / dt:.0f} inserts/s ({dt:.2f} s), insert kernels {st['build_search_us'] / 1e6:.3f} s, "
          f"evals/insert {st['build_dist_evals'] / n:.0f}; " + "; ".join(out), flush=True)
    g.close()
