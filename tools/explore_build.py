import sys, time, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np, torch
import hnsw_amd as H
from bench import gen_vectors

def clustered(rng, n, d, nc=64, intrinsic=12, noise=0.05):
    C = rng.normal(size=(nc, intrinsic)).astype(np.float32)
    A = rng.normal(size=(intrinsic, d)).astype(np.float32) / np.sqrt(intrinsic)
    z = C[rng.integers(0, nc, n)] + 0.35 * rng.normal(size=(n, intrinsic)).astype(np.float32)
    return (z @ A + noise * rng.normal(size=(n, d)).astype(np.float32)).astype(np.float32)

def run(X, Q, metric, **kw):
    ef_search = kw.pop("ef_search", 64)
    g = H.Graph(M=kw.pop("M", 16), Ml=0.25, EfSearch=ef_search, Distance=metric, Rng=9, build_mode=H.BUILD_BATCH, **kw)
    Xt = torch.from_numpy(X).cuda() if isinstance(X, np.ndarray) else X
    torch.cuda.synchronize(); t0 = time.time()
    g.add_device(np.arange(Xt.shape[0]), Xt.data_ptr(), Xt.shape[0], Xt.shape[1])
    torch.cuda.synchronize(); bt = time.time() - t0
    Qn = Q if isinstance(Q, np.ndarray) else Q.cpu().numpy()
    ek, ed, en = g.search_arrays(Qn, 10, mode=H.MODE_EXACT)
    out = []
    for ef in (32, 64, 128):
        bk, bd, bn = g.search_arrays(Qn, 10, mode=H.MODE_BEAM, ef=ef)
        r = np.mean([len(set(bk[b, :bn[b]]) & set(ek[b, :en[b]])) / 10 for b in range(len(Qn))])
        out.append(round(r, 4))
    st = g.stats()
    return bt, out, st

dev = torch.device("cuda")
import itertools
def run2(X, Q, **kw):
    g = H.Graph(M=kw.pop("M", 16), Ml=0.25, EfSearch=64, Distance=H.CosineDistance, Rng=9, build_mode=H.BUILD_BATCH, **kw)
    torch.cuda.synchronize(); t0 = time.time()
    g.add_device(np.arange(X.shape[0]), X.data_ptr(), X.shape[0], X.shape[1])
    torch.cuda.synchronize(); bt = time.time() - t0
    Qn = Q.cpu().numpy()
    ek, ed, en = g.search_arrays(Qn, 10, mode=H.MODE_EXACT)
    out = []
    for ef in (32, 64, 128, 256):
        bk, bd, bn = g.search_arrays(Qn, 10, mode=H.MODE_BEAM, ef=ef)
        out.append(round(float(np.mean([len(set(bk[b, :bn[b]]) & set(ek[b, :en[b]])) / 10 for b in range(len(Qn))])), 4))
    return bt, out
n = 1000000
for intr in (8, 12, 16):
    X = gen_vectors(n, 768, 1234, intr, 1000, dev, "cosine")
    Q = gen_vectors(500, 768, 99, intr, 1000, dev, "cosine")
    for kw in [dict(ef_construction=200, m0=48, heuristic=2), dict(ef_construction=200, m0=48, heuristic=2, batch_ratio_pct=1, batch_max=8192)]:
        bt, r = run2(X, Q, **dict(kw))
        print("intrinsic", intr, kw, "build %.2fs" % bt, "recall@ef32/64/128/256", r, flush=True)
    del X
