"""Config-5 exact-path probe for kernel profiling: 1M x 1536 cosine, batch 1024,
a flat index (vector store only), `reps` exact searches.
Usage: python tools/exact_probe.py [precision=1] [tile=0] [reps=3]"""
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import hnsw_amd as H  # noqa: E402
from bench import Searcher, gen_vectors  # noqa: E402

prec = int(sys.argv[1]) if len(sys.argv) > 1 else 1
tile = int(sys.argv[2]) if len(sys.argv) > 2 else 0
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
dev = torch.device("cuda")
n, d, B = 1_000_000, 1536, 1024
X = gen_vectors(n, d, 55, 12, 1000, dev, "cosine")
Q = gen_vectors(B, d, 56, 12, 1000, dev, "cosine")
g = H.Graph(M=4, Ml=0.25, EfSearch=8, Distance=H.CosineDistance, Rng=5, build_mode=H.BUILD_FLAT)
g.reserve(n, d)
torch.cuda.synchronize()
g.add_device(np.arange(n), X.data_ptr(), n, d)
del X
g.set_option("exact_precision", prec)
g.set_option("exact_tile", tile)
if os.environ.get("EXACT_SAMPLE"):
    g.set_option("exact_sample", int(os.environ["EXACT_SAMPLE"]))
if os.environ.get("EXACT_THR_RANK"):
    g.set_option("exact_thr_rank", int(os.environ["EXACT_THR_RANK"]))
S = Searcher(g, B, 10, d, dev)


def run():
    try:
        S.run(Q, H.MODE_EXACT, 0)
    except H.HnswError as e:  # exact_tile 30-32, 36-39 (MHNSW_LIB=tools/libmhnsw_diag.so): no results
        if tile not in (30, 31, 32, 36, 37, 38, 39, 41):
            raise
        assert "timing diagnostic" in str(e)


run()
torch.cuda.synchronize()
g.reset_stats()
t0 = time.perf_counter()
for _ in range(reps):
    run()
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / reps
print(f"precision={prec} tile={tile} thr_rank={g.get_option('exact_thr_rank')} ms_per_batch={dt * 1e3:.3f} "
      f"uncertified={g.stats().get('exact_uncertified')}", flush=True)
