"""Where the layer-0 beam's shader cycles go (tools-only build with MH_PROF_BEAM:
  make -C tools -f Makefile.beam TAG=pbeam BFLAGS=-DMH_PROF_BEAM
run with MHNSW_LIB=tools/libmhnsw_pbeam.so): cycles per query in list insertions
(bl_insert), in candidate scoring (screen + f32, without the insertions), and in
the whole layer-0 search, on the harder-data graph (bench.config_harder's) at
the given (search_expand, ef) points.
Usage: python tools/beam_cycles_probe.py [XW:EF ...]   (default 4:496 1:496 4:256 1:64)"""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import hnsw_amd as H  # noqa: E402
from bench import Searcher, gen_vectors  # noqa: E402

dev = torch.device("cuda")
n, d, B = 1_000_000, 768, 16384
X = gen_vectors(n, d, 4321, 32, 1000, dev, "cosine")
Q = gen_vectors(B, d, 4321 + 7777, 32, 1000, dev, "cosine")
g = H.Graph(M=32, Ml=0.25, EfSearch=64, Distance=H.CosineDistance, Rng=5, build_mode=H.BUILD_BATCH, m0=63,
            ef_construction=512, heuristic=2, keep_pruned=1, prune_alpha_pct=115, build_expand=4, screen=1,
            batch_ratio_pct=20)
g.reserve(n, d)
g.add_device(np.arange(n), X.data_ptr(), n, d)
del X
S = Searcher(g, B, 10, d, dev)
pts = [tuple(int(v) for v in a.split(":")) for a in sys.argv[1:]] or [(4, 496), (1, 496), (4, 256), (1, 64)]
for xw, ef in pts:
    g.set_option("search_expand", xw)
    S.run(Q, H.MODE_BEAM, ef)
    g.reset_stats()
    S.run(Q, H.MODE_BEAM, ef)
    ms = g.last_kernel_ms()
    st = g.stats()
    ins, sc, al = st["build_screened"] / B, st["build_f32_rows"] / B, st["exact_uncertified"] / B
    print(f"XW {xw} ef {ef}: kernel {ms:.3f} ms; per query: layer-0 cycles {al:,.0f}, insertions {ins:,.0f} "
          f"({ins / al:.1%}), scoring {sc:,.0f} ({sc / al:.1%}), rest {al - ins - sc:,.0f} ({(al - ins - sc) / al:.1%}); "
          f"screened {st['search_screened'] / B:.0f}, f32 {st['search_f32_evals'] / B:.0f}, "
          f"expansions {st['search_expansions'] / B:.0f}", flush=True)
