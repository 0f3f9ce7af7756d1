"""Batched-insert schedule probe on the bench index (bench.py defaults: 1M x
768 cosine latent 12, M 16, M0 40, efC 400, heuristic 2, keep-pruned fill,
slack 1.15): build time and recall@10 at ef 64 (4,096 queries vs the exact
path) per batch schedule.  A batch of b new nodes is searched against the
graph as it stood before the batch, so the schedule (batch_min, batch_ratio_pct,
batch_max) trades early-phase launches for within-batch links.
Usage: BUILD_OPTS="batch_min=1;batch_min=256,batch_ratio_pct=10" python tools/schedule_probe.py
   or: python tools/schedule_probe.py "batch_min=1;batch_min=256+batch_ratio_pct=10"""
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
# CFG2=1: BASELINE configs[2] instead (1M x 768 Euclidean, M0 48, efC 64, closest-M fill off; bench.py config2)
cfg2 = os.environ.get("CFG2", "0") == "1"
hard = os.environ.get("HARD", "0") == "1"  # the harder-data leg (latent 32, M 32, M0 63, efC 512)
efs = (256, 512) if hard else (48, 64)
if os.environ.get("EFS"):  # e.g. EFS=320+384+448+512
    efs = tuple(int(x) for x in os.environ["EFS"].split("+"))
if hard:
    X = gen_vectors(n, d, 4321, 32, 1000, dev, "cosine")
    Q = gen_vectors(4096, d, 4321 + 7777, 32, 1000, dev, "cosine")
    base = dict(Distance=H.CosineDistance, Rng=5, m0=63, ef_construction=512, heuristic=2, keep_pruned=1,
                prune_alpha_pct=115, build_expand=2, M=32)
elif cfg2:
    X = gen_vectors(n, d, 77, 12, 1000, dev, "euclidean")
    Q = gen_vectors(4096, d, 78, 12, 1000, dev, "euclidean")
    base = dict(Distance=H.EuclideanDistance, Rng=5, m0=48, ef_construction=64, heuristic=2)
else:
    X = gen_vectors(n, d, 1234, 12, 1000, dev, "cosine")
    Q = gen_vectors(4096, d, 1234 + 7777, 12, 1000, dev, "cosine")
    base = dict(Distance=H.CosineDistance, Rng=1234, m0=40, ef_construction=400, heuristic=2, keep_pruned=1,
                prune_alpha_pct=115)
# option sets: BUILD_OPTS, or argv[1] with "+" between one set's options (tools/gpu_run.sh splits steps at commas)
spec = sys.argv[1].replace("+", ",") if len(sys.argv) > 1 else os.environ.get("BUILD_OPTS", "")
sets = [dict(kv.split("=") for kv in s_.split(",") if kv) for s_ in spec.split(";")]
truth = None
for opts in sets:
    kw = dict(base)
    kw.update({k: int(v) for k, v in opts.items()})
    kw.setdefault("M", 16)
    g = H.Graph(Ml=0.25, EfSearch=64, build_mode=H.BUILD_BATCH, **kw)
    g.reserve(n, d)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g.add_device(np.arange(n), X.data_ptr(), n, d)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if truth is None:
        truth = tuple(x.clone() for x in Searcher(g, 4096, 10, d, dev).run(Q, H.MODE_EXACT, 0))
    S = Searcher(g, 4096, 10, d, dev)
    recs = []
    for ef in efs:
        k_, _, n_ = S.run(Q, H.MODE_BEAM, ef)
        recs.append(recall_at_k(k_, n_, truth[0], truth[2], 10))
    print(f"{opts}: {n / dt:.0f} inserts/s ({dt:.2f} s), recall@10 " +
          " ".join(f"ef{e} {r:.4f}" for e, r in zip(efs, recs)), flush=True)
    g.close()
