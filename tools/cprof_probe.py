"""Reference-semantics insert (compat Add) cycle accounting on the configs[0]
shape (10k x 128 U[-1,1) cosine, M 16, Ml 0.25, EfSearch 20): run with
MHNSW_LIB=tools/libmhnsw_cprof.so (tools/Makefile.build TAG=cprof
BFLAGS=-DMH_COMPAT_PROF); the kernel prints `cprof <slot> <cycles>` lines.
Usage: python tools/cprof_probe.py [n] [d] [waves]"""
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import hnsw_amd as H  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000
d = int(sys.argv[2]) if len(sys.argv) > 2 else 128
waves = int(sys.argv[3]) if len(sys.argv) > 3 else 8
rng = np.random.default_rng(42)
X = rng.uniform(-1, 1, (n, d)).astype(np.float32)
g = H.Graph(M=16, Ml=0.25, EfSearch=20, Distance=H.CosineDistance, Rng=42, compat_waves=waves)
torch.cuda.synchronize()
t0 = time.perf_counter()
g.add_arrays(np.arange(n), X)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
st = g.stats()
print(f"compat add n={n} d={d} waves={waves}: {n / dt:.1f} inserts/s, {st['build_dist_evals'] / n:.0f} dist evals/insert, "
      f"{st['build_expansions'] / n:.0f} expansions/insert", flush=True)
