"""GPU parity at BASELINE.json's full sizes, against the oracle on the same
graph, plus size-independent properties:

  configs[1]  1M x 768 cosine graph (the bench.py index): the engine's beam
              result lists (keys, counts, distance bits) == the oracle's beam
              search (graph.go:1047-1110 BatchSearch loop, ORDER_DEV) on the
              exported graph for all 2048 queries, and its exact lists == the
              oracle's brute force on 64 of them; the fp16 screen never changes
              a result (screen on == off, bitwise); lists sorted, keys unique;
              self-queries find themselves; beam recall vs the exact path.
              The reference's Search() semantics (k_search_compat,
              graph.go:534-625) on the same 1M graph == the oracle's compat
              Search (ORDER_DEV) on 2048 queries, bitwise.  Against the
              reference's arithmetic (ORDER_REF, sequential fp32): beam and
              compat recall@10 within 0.002, distances within 1e-5.
  configs[2]  1M x 768 Euclidean batched insert (efConstruction 64): a
              well-formed graph (ids in range, no self loops, sets, degree
              caps), beam lists == the oracle's on 1024 queries, exact == the
              oracle's brute force on 32, recall@10 >= 0.99 at ef 64.
  configs[4]  1M x 1536 cosine exact path, batch 1024: every precision
              certifies to the same results, == the oracle's brute force
              (keys + distance bits) on 32 queries, self-queries first.
The oracle runs multi-threaded on the host's usable cores (bench.host_threads,
the same concurrent Search as graph_benchmark_test.go:70-89).  Vectors come
from bench.gen_vectors."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _gen(n, d, seed, metric):
    from bench import gen_vectors

    return gen_vectors(n, d, seed, 12, 1000, torch.device("cuda"), metric)


def _search(g, Q, k, mode, ef):
    from bench import Searcher

    S = Searcher(g, Q.shape[0], k, Q.shape[1], torch.device("cuda"))
    return [x.clone().cpu().numpy() for x in S.run(Q, mode, ef)]


def _threads():
    from bench import host_threads

    return max(1, min(64, host_threads()))


def _oracle_of(O, g, metric, M, M0, ef):
    """the engine's graph exported (rows, layers, adjacency, entries) into the
    oracle, which then searches it with the reference's algorithm"""
    o = O.Graph(metric=metric, order=O.ORDER_DEV, M=M, M0=M0, Ml=0.25, EfSearch=ef)
    o.import_graph(**g.export())
    return o


def _same_lists(got, want, tag):
    gk, gd, gn = got
    rk, rd, rn = want
    assert np.array_equal(gn, rn), tag
    for b in range(len(gn)):
        m = gn[b]
        assert np.array_equal(gk[b, :m], rk[b, :m]), (tag, b)
        assert np.array_equal(gd[b, :m].view(np.uint32), rd[b, :m].view(np.uint32)), (tag, b)


def _check_lists(keys, dist, n, N):
    for b in range(len(n)):
        kb, db = keys[b, : n[b]], dist[b, : n[b]]
        assert len(set(kb.tolist())) == len(kb), b
        assert ((kb >= 0) & (kb < N)).all(), b
        assert np.all(db[1:] >= db[:-1]), b


def _check_oracle_distances(O, metric, X, Q, keys, n, rows=128):
    """the reported distance of (query, result) pairs == the oracle's canonical one, bitwise"""
    sel = np.arange(0, len(n), max(1, len(n) // rows))[:rows]
    for b in sel:
        kb = keys[b, : n[b]]
        xs = X[torch.from_numpy(kb).to(X.device)].cpu().numpy()
        q = Q[b].cpu().numpy()
        want = np.array([O.distance(metric, O.ORDER_DEV, x, q) for x in xs], np.float32)
        yield b, want


def test_fullsize_c2_beam(H, O):
    n, d, B = 1_000_000, 768, 2048
    X = _gen(n, d, 1234, "cosine")
    Q = _gen(B, d, 1234 + 7777, "cosine")
    g = H.Graph(M=16, Ml=0.25, EfSearch=64, Distance=H.CosineDistance, Rng=1234, build_mode=H.BUILD_BATCH, m0=40,
                ef_construction=400, heuristic=2, keep_pruned=1, prune_alpha_pct=115)
    g.reserve(n, d)
    g.add_device(np.arange(n), X.data_ptr(), n, d)
    assert len(g) == n and g.stats()["dropped_proposals"] == 0
    on = _search(g, Q, 10, H.MODE_BEAM, 64)
    g.set_option("screen", 0)
    off = _search(g, Q, 10, H.MODE_BEAM, 64)
    assert np.array_equal(on[2], off[2]) and np.array_equal(on[0], off[0])
    assert np.array_equal(on[1].view(np.uint32), off[1].view(np.uint32))
    g.set_option("screen", 1)
    keys, dist, cnt = on
    assert (cnt == 10).all()
    _check_lists(keys, dist, cnt, n)
    for b, want in _check_oracle_distances(O, 0, X, Q, keys, cnt):
        assert np.array_equal(dist[b, : cnt[b]].view(np.uint32), want.view(np.uint32)), b
    ek, ed, en = _search(g, Q, 10, H.MODE_EXACT, 0)
    _check_lists(ek, ed, en, n)
    rec = np.mean([len(set(keys[b]) & set(ek[b, : en[b]])) / 10 for b in range(B)])
    assert rec >= 0.98, rec
    # the oracle's BatchSearch on the same graph: every list identical
    o = _oracle_of(O, g, O.COSINE, 16, 40, 64)
    Qh = Q.cpu().numpy()
    _same_lists(on, o.search(Qh, 10, mode=O.MODE_BEAM, ef=64, threads=_threads()), "beam")
    sub = np.arange(0, B, B // 64)[:64]
    _same_lists((ek[sub], ed[sub], en[sub]), o.search(Qh[sub], 10, mode=O.MODE_EXACT, threads=_threads()), "exact")
    # the reference's Search() semantics on the 1M graph (graph.go:534-625), bitwise
    ck = _search(g, Q, 10, H.MODE_COMPAT, 64)
    g.device_status()
    _same_lists(ck, o.search(Qh, 10, mode=O.MODE_COMPAT, ef=64, threads=_threads()), "compat")
    # the north-star criterion against the reference's arithmetic (ORDER_REF)
    from oracle.parity import compare_lists

    o.set_order(O.ORDER_REF)
    for tag, got, mode in (("beam", on, O.MODE_BEAM), ("compat", ck, O.MODE_COMPAT)):
        pr = compare_lists(got, o.search(Qh, 10, mode=mode, ef=64, threads=_threads()), 10, truth=(ek, en))
        print(f"configs[1] GPU {tag} vs ORDER_REF:", pr)
        assert pr["recall_delta"] <= 0.002 and pr["max_abs_dist_diff"] <= 1e-5, (tag, pr)
    del o
    # self-queries: a stored row finds itself first (distance 0 or the -1.19e-7 of parallel vectors)
    ids = np.random.default_rng(5).choice(n, 512, replace=False)
    sk, sd, sn = _search(g, X[torch.from_numpy(ids).cuda()].contiguous(), 10, H.MODE_BEAM, 64)
    assert (sk[:, 0] == ids).mean() >= 0.99
    assert np.all(np.abs(sd[:, 0][sk[:, 0] == ids]) <= 2.5e-7)
    g.close()


def test_fullsize_c3_build(H, O):
    n, d, B = 1_000_000, 768, 1024
    X = _gen(n, d, 77, "euclidean")
    Q = _gen(B, d, 78, "euclidean")
    g = H.Graph(M=16, Ml=0.25, EfSearch=64, Distance=H.EuclideanDistance, Rng=5, build_mode=H.BUILD_BATCH, m0=48,
                ef_construction=64, heuristic=2)
    g.reserve(n, d)
    g.add_device(np.arange(n), X.data_ptr(), n, d)
    assert g.stats()["dropped_proposals"] == 0
    ex = g.export()
    deg, adj = ex["deg"], ex["adj"]
    L, N, cap = adj.shape
    assert N == n
    for l in range(L):
        dl = deg[l]
        assert (dl >= -2).all() and (dl < cap).all()
        rows = np.nonzero(dl > 0)[0]
        for i in rows[:: max(1, len(rows) // 20000)]:  # sampled rows: ids in range, no self loops, sets
            r = adj[l, i, : dl[i]]
            assert ((r >= 0) & (r < n)).all() and (r != i).all() and len(set(r.tolist())) == len(r), (l, i)
            assert (deg[l, r] != -2).all(), (l, i)  # every neighbour is a member of the layer
    assert (deg[0] >= 1).all()
    bk, bd, bn = _search(g, Q, 10, H.MODE_BEAM, 64)
    ek, ed, en = _search(g, Q, 10, H.MODE_EXACT, 0)
    _check_lists(bk, bd, bn, n)
    rec = np.mean([len(set(bk[b, : bn[b]]) & set(ek[b, : en[b]])) / 10 for b in range(B)])
    assert rec >= 0.99, rec
    o = _oracle_of(O, g, O.EUCLIDEAN, 16, 48, 64)
    Qh = Q.cpu().numpy()
    _same_lists((bk, bd, bn), o.search(Qh, 10, mode=O.MODE_BEAM, ef=64, threads=_threads()), "beam")
    sub = np.arange(0, B, B // 32)[:32]
    _same_lists((ek[sub], ed[sub], en[sub]), o.search(Qh[sub], 10, mode=O.MODE_EXACT, threads=_threads()), "exact")
    del o
    g.close()


def test_fullsize_c5_exact(H, O):
    n, d, B = 1_000_000, 1536, 1024
    X = _gen(n, d, 55, "cosine")
    Q = _gen(B, d, 56, "cosine")
    ids = np.arange(0, n, n // 16)[:16]
    Q[:16] = X[torch.from_numpy(ids).cuda()]  # self-queries
    g = H.Graph(M=16, Ml=0.25, EfSearch=64, Distance=H.CosineDistance, Rng=5, build_mode=H.BUILD_FLAT)
    g.reserve(n, d)
    g.add_device(np.arange(n), X.data_ptr(), n, d)
    res = {}
    for prec in (0, 1, 2, 3):
        g.set_option("exact_precision", prec)
        g.reset_stats()
        res[prec] = _search(g, Q, 10, H.MODE_EXACT, 0)
        if prec == 3:  # the fused preselection certifies (nearly) every query without the sweep
            assert g.stats()["exact_uncertified"] <= 8, g.stats()
    for p in (1, 2, 3):
        for a, b in zip(res[0], res[p]):
            assert np.array_equal(np.asarray(a).view(np.uint8), np.asarray(b).view(np.uint8)), p
    keys, dist, cnt = res[1]
    assert (cnt == 10).all()
    _check_lists(keys, dist, cnt, n)
    assert (keys[:16, 0] == ids).all()
    for b, want in _check_oracle_distances(O, 0, X, Q, keys, cnt, rows=64):
        assert np.array_equal(dist[b, : cnt[b]].view(np.uint32), want.view(np.uint32)), b
    # the oracle's brute force (every row, canonical distances) on 32 queries, 16 of them self-queries
    del X
    o = _oracle_of(O, g, O.COSINE, 16, 16, 64)
    sub = np.concatenate([np.arange(8), np.arange(16, B, (B - 16) // 24)[:24]])
    want = o.search(Q.cpu().numpy()[sub], 10, mode=O.MODE_EXACT, threads=_threads())
    del o
    for p in (0, 3):
        _same_lists(tuple(np.asarray(x)[sub] for x in res[p]), want, ("exact", p))
    g.close()


@pytest.mark.parametrize("tile", [34, 5])
@pytest.mark.parametrize("metric,k", [("cosine", 10), ("cosine", 256), ("l2", 64)])
def test_exact_record_variants(H, O, tile, metric, k):
    """Both precision-3 GEMM variants -- k_h1_pp16 with the record-mode fused
    filter (34, the default) and the ring kernel's pair filter (5, the fallback
    for shapes the stream does not admit) -- certify to the f32-input results
    bitwise.  Ragged row and query tiles; k = 256 widens the threshold."""
    n, d, B = 300_007, 1536, 700
    X = _gen(n, d, 57, metric)
    Q = _gen(B, d, 58, metric)
    dist = H.CosineDistance if metric == "cosine" else H.EuclideanDistance
    g = H.Graph(M=16, Ml=0.25, EfSearch=64, Distance=dist, Rng=5, build_mode=H.BUILD_FLAT)
    g.reserve(n, d)
    g.add_device(np.arange(n), X.data_ptr(), n, d)
    g.set_option("exact_precision", 0)
    ref = _search(g, Q, k, H.MODE_EXACT, 0)
    g.set_option("exact_precision", 3)
    g.set_option("exact_tile", tile)
    g.reset_stats()
    got = _search(g, Q, k, H.MODE_EXACT, 0)
    for a, b in zip(ref, got):
        assert np.array_equal(np.asarray(a).view(np.uint8), np.asarray(b).view(np.uint8)), tile
    assert (got[2] == k).all()
    g.close()


@pytest.mark.parametrize("metric,k,rank", [("cosine", 10, 10), ("l2", 64, 16), ("cosine", 1, 1)])
def test_exact_threshold_rank(H, O, metric, k, rank):
    """A lower threshold rank (exact_thr_rank: the sample's J-th best, J >= k)
    passes fewer pairs through the fused filter; results stay bit-identical to
    the f32-input exact path (certified, or redone by the canonical sweep)."""
    n, d, B = 200_003, 1536, 513
    X = _gen(n, d, 61, metric)
    Q = _gen(B, d, 62, metric)
    dist = H.CosineDistance if metric == "cosine" else H.EuclideanDistance
    g = H.Graph(M=16, Ml=0.25, EfSearch=64, Distance=dist, Rng=5, build_mode=H.BUILD_FLAT)
    g.reserve(n, d)
    g.add_device(np.arange(n), X.data_ptr(), n, d)
    g.set_option("exact_precision", 0)
    ref = _search(g, Q, k, H.MODE_EXACT, 0)
    g.set_option("exact_precision", 3)
    g.set_option("exact_thr_rank", rank)
    got = _search(g, Q, k, H.MODE_EXACT, 0)
    for a, b in zip(ref, got):
        assert np.array_equal(np.asarray(a).view(np.uint8), np.asarray(b).view(np.uint8)), rank
    g.close()


@pytest.mark.parametrize("metric", ["cosine", "l2"])
def test_exact_fused_fallback_segments(H, O, metric):
    """kk = k leaves the certificate no margin, so (nearly) every query takes the
    fallback.  On the fused fp16 path it streams canonical distances into
    per-segment lists (k_fallback_select: 16 segments x 4 waves per query, no
    score matrix); the results equal the f32-input path's (whose fallback writes
    a score row per query), bitwise, with deleted rows and a ragged row count."""
    n, d, B, k = 200_003, 768, 96, 10
    X = _gen(n, d, 63, metric)
    Q = _gen(B, d, 64, metric)
    dist = H.CosineDistance if metric == "cosine" else H.EuclideanDistance
    g = H.Graph(M=16, Ml=0.25, EfSearch=64, Distance=dist, Rng=5, build_mode=H.BUILD_FLAT)
    g.reserve(n, d)
    g.add_device(np.arange(n), X.data_ptr(), n, d)
    g.BatchDelete([int(x) for x in np.random.default_rng(3).choice(n, 2000, replace=False)])
    g.set_option("exact_kk", k)
    res = {}
    for prec in (0, 3):
        g.set_option("exact_precision", prec)
        g.reset_stats()
        res[prec] = _search(g, Q, k, H.MODE_EXACT, 0)
        assert g.stats()["exact_uncertified"] >= B // 2, (prec, g.stats())
    for a, b in zip(res[0], res[3]):
        assert np.array_equal(np.asarray(a).view(np.uint8), np.asarray(b).view(np.uint8))
    assert (res[3][2] == k).all()
    g.close()
