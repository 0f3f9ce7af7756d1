"""Small-batch latency probe on the bench graph (1M x 768 cosine, bench.py
defaults): ms per batch of B queries at ef 64 with the one-wave kernel
(beam_mw_max_b 0) and the 4-wave small-batch kernel (beam_mw_max_b large),
to place the switch-over.  Usage: python tools/batch_probe.py [B list]"""
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import hnsw_amd as H  # noqa: E402
from bench import Searcher, gen_vectors  # noqa: E402

dev = torch.device("cuda")
n, d = 1_000_000, 768
bs = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1,16,64,256,512,1024,2048,4096").split(",")]
X = gen_vectors(n, d, 1234, 12, 1000, dev, "cosine")
Q = gen_vectors(max(bs), d, 1234 + 7777, 12, 1000, dev, "cosine")
g = H.Graph(M=16, Ml=0.25, EfSearch=64, Distance=H.CosineDistance, Rng=1234, build_mode=H.BUILD_BATCH, m0=40,
            ef_construction=400, heuristic=2, keep_pruned=1, prune_alpha_pct=115)
g.reserve(n, d)
g.add_device(np.arange(n), X.data_ptr(), n, d)
del X
modes = [(0, 1), (1 << 30, 1)]
if os.environ.get("SCREEN_OFF") == "1":  # also the 4-wave kernel without the fp16 screen
    modes.append((1 << 30, 0))
for B in bs:
    S = Searcher(g, B, 10, d, dev)
    row = []
    for mw, scr in modes:
        g.set_option("beam_mw_max_b", mw)
        if g.get_option("screen") != scr:
            g.set_option("screen", scr)
        reps = max(5, min(400, 40000 // B))
        S.run(Q[:B], H.MODE_BEAM, 64)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            S.run(Q[:B], H.MODE_BEAM, 64)
        torch.cuda.synchronize()
        row.append((time.perf_counter() - t0) / reps * 1e3)
    extra = f" four_wave_noscreen_ms={row[2]:.4f}" if len(row) > 2 else ""
    print(f"B={B} one_wave_ms={row[0]:.4f} four_wave_ms={row[1]:.4f} ratio={row[0] / row[1]:.3f}{extra}", flush=True)
    if len(row) > 2:
        g.set_option("screen", 1)
g.close()
