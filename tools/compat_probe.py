"""Reference-semantics insert (compat build, graph.go:437-531) throughput probe:
n x d Euclidean, M=16, EfSearch=20, one wave walking the inserts in order.
Usage: python tools/compat_probe.py [n] [d]"""
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import hnsw_amd as H  # noqa: E402
from bench import gen_vectors  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
d = int(sys.argv[2]) if len(sys.argv) > 2 else 768
waves = int(sys.argv[3]) if len(sys.argv) > 3 else 8
dev = torch.device("cuda")
X = gen_vectors(n, d, 77, 12, 1000, dev, "euclidean")
g = H.Graph(M=16, Ml=0.25, EfSearch=20, Distance=H.EuclideanDistance, Rng=5, compat_waves=waves)
g.reserve(n, d)
torch.cuda.synchronize()
t0 = time.perf_counter()
g.add_device(np.arange(n), X.data_ptr(), n, d)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
st = g.stats()
print(f"compat insert n={n} d={d} waves={waves}: {n / dt:.1f} inserts/s, {st['build_dist_evals'] / n:.0f} dist evals/insert, "
      f"{st['build_expansions'] / n:.0f} expansions/insert", flush=True)
