"""Feasibility probe (tools only): how many of a beam search's candidates could a
projection lower bound reject?  For cosine rows (unit vectors) d = |q - x|^2 / 2 and an
orthonormal projection P gives |P(q - x)|^2 / 2 <= d.  On the bench index (and the
harder latent-32 data), for 256 queries: the exact top-64's worst distance w, the
candidates a converged beam meets (the layer-0 rows of the exact top-64, minus them),
and the fraction of those with d > w (what any exact screen may reject) and with
LB_k > w for PCA projections of k dims.  Usage: python tools/proj_probe.py [latent ...]"""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import hnsw_amd as H  # noqa: E402
from bench import gen_vectors  # noqa: E402

dev = torch.device("cuda")
n, d, nq = 1_000_000, 768, 256
for latent in [int(a) for a in sys.argv[1:]] or [12]:
    seed = 1234 if latent == 12 else 4321
    X = gen_vectors(n, d, seed, latent, 1000, dev, "cosine")
    Q = gen_vectors(nq, d, seed + 7777, latent, 1000, dev, "cosine")
    kw = dict(M=16, m0=40, ef_construction=400, upper_efc=128) if latent == 12 else dict(M=32, m0=63, ef_construction=512, upper_efc=256)
    M = kw.pop("M")
    g = H.Graph(M=M, Ml=0.25, EfSearch=64, Distance=H.CosineDistance, Rng=seed, build_mode=H.BUILD_BATCH, heuristic=2,
                keep_pruned=1, prune_alpha_pct=115, build_expand=4, batch_ratio_pct=20, **kw)
    g.reserve(n, d)
    g.add_device(np.arange(n), X.data_ptr(), n, d)
    ex = g.export()
    g.close()
    deg0 = torch.from_numpy(ex["deg"][0]).to(dev)
    adj0 = torch.from_numpy(ex["adj"][0]).to(dev)
    del ex
    D = 1.0 - Q @ X.T  # [nq, n]
    for ef in (64, 512):
        top = torch.topk(D, ef, dim=1, largest=False)
        w = top.values[:, -1]
        sel = torch.randperm(n, device=dev)[:100_000]
        Xs = X[sel]
        C = (Xs.T @ Xs) / Xs.shape[0]
        evals, evecs = torch.linalg.eigh(C.double())
        evecs = evecs.float().flip(1)
        stats = {"d>w": []}
        ks = (8, 16, 32, 64, 128)
        for k in ks:
            stats[k] = []
        for b in range(nq):
            ids = top.indices[b]
            rows = adj0[ids]
            msk = torch.arange(adj0.shape[1], device=dev)[None, :] < deg0[ids][:, None]
            cand = torch.unique(rows[msk])
            cand = cand[(cand >= 0)]
            cand = cand[~torch.isin(cand, ids)]
            dc = D[b, cand]
            stats["d>w"].append((dc > w[b]).float().mean().item())
            diff = Q[b][None, :] - X[cand]
            for k in ks:
                P = evecs[:, :k]
                lb = (diff @ P).pow(2).sum(1) / 2
                stats[k].append((lb > w[b] * 1.0005 + 1e-6).float().mean().item())
        var = evals.flip(0).float()
        print(f"latent {latent} ef {ef}: candidates/query ~{len(cand)}, exact screen could reject "
              f"{np.mean(stats['d>w']):.3f}; projection LB rejects " +
              ", ".join(f"k={k}: {np.mean(stats[k]):.3f}" for k in ks) +
              f"; variance in top 16/32/64 dims {var[:16].sum() / var.sum():.3f}/{var[:32].sum() / var.sum():.3f}/"
              f"{var[:64].sum() / var.sum():.3f}", flush=True)
    del X, D
    torch.cuda.empty_cache()
