"""Batched-insert probe (BASELINE configs[2]: 1M x 768 Euclidean, M=16, M0=48,
heuristic 2): inserts/s and per-insert counters for each efConstruction given.
Usage: python tools/build_probe.py [efc ...]"""
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import hnsw_amd as H  # noqa: E402
from bench import gen_vectors  # noqa: E402

dev = torch.device("cuda")
n = int(os.environ.get("BUILD_N", 1_000_000))
# BUILD_BENCH=1: the bench index instead (cosine, M0 40, keep-pruned fill, slack 1.15; bench.py defaults)
bench_cfg = os.environ.get("BUILD_BENCH", "0") == "1"
if bench_cfg:
    X = gen_vectors(n, 768, 1234, 12, 1000, dev, "cosine")
    base = dict(Distance=H.CosineDistance, Rng=1234, m0=40, keep_pruned=1, prune_alpha_pct=115)
else:
    X = gen_vectors(n, 768, 77, 12, 1000, dev, "euclidean")
    base = dict(Distance=H.EuclideanDistance, Rng=5, m0=48)
# BUILD_OPTS="a=1,b=2;a=3": one build per ';'-separated option set
sets = [dict(kv.split("=") for kv in s_.split(",") if kv) for s_ in os.environ.get("BUILD_OPTS", "").split(";")]
for efc, opts in [(e, o) for e in ([int(a) for a in sys.argv[1:]] or [64]) for o in sets]:
    kw = dict(base, heuristic=2)
    kw.update({k: int(v) for k, v in opts.items()})
    g = H.Graph(M=16, Ml=0.25, EfSearch=64, build_mode=H.BUILD_BATCH, ef_construction=efc, **kw)
    g.reserve(n, 768)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g.add_device(np.arange(n), X.data_ptr(), n, 768)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st = g.stats()
    print(f"efc={efc} {opts}: {n / dt:.0f} inserts/s ({dt:.2f} s), {st['build_dist_evals'] / n:.0f} evals/insert, "
          f"{st['build_expansions'] / n:.0f} expansions/insert, screened {st['build_screened'] / n:.0f}, "
          f"f32 {st['build_f32_rows'] / n:.0f}, insert kernels {st['build_search_us'] / 1e6:.2f} s, "
          f"dropped {st['dropped_proposals']}", flush=True)
    g.close()
