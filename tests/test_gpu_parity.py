"""GPU parity: the HIP engine (through the C ABI) against the CPU restatement
(oracle/) on identical inputs.  Integer/index results must be identical;
distances must be bit-identical to the oracle's canonical-order restatement
(OG_ORDER_DEV) and within 1e-5 (relative for L2) of the sequential-fp32
restatement of vek32 (OG_ORDER_REF)."""
import json
import os
import struct

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
TOL = 1e-5  # north_star: distances within 1e-5 fp32


def _bits(x):
    return struct.unpack("<I", struct.pack("<f", float(x)))[0]


def _levels(O, metric, M, ml, ef, seed, n):
    g = O.Graph(metric=metric, order=O.ORDER_DEV, M=M, Ml=ml, EfSearch=ef, seed=seed)
    return g.preview_levels(n)


def _metric_fn(H, metric):
    return H.CosineDistance if metric == 0 else H.EuclideanDistance


def _bit_equal(a, b):
    """bitwise equality, any NaN equal to any NaN (NaN sign/payload is not meaningful)"""
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    na, nb = np.isnan(a), np.isnan(b)
    return np.array_equal(na, nb) and np.array_equal(a[~na].view(np.uint32), b[~nb].view(np.uint32))


def _same_graph(a, b):
    assert np.array_equal(a["keys"], b["keys"])
    assert np.array_equal(a["deg"], b["deg"]), "degree arrays differ"
    L, N = a["deg"].shape
    for l in range(L):
        for i in range(N):
            d = a["deg"][l, i]
            if d > 0:
                assert set(a["adj"][l, i, :d].tolist()) == set(b["adj"][l, i, :d].tolist()), (l, i)
    assert np.array_equal(a["entry"], b["entry"])
    if "dead" in a and "dead" in b:
        assert np.array_equal(a["dead"], b["dead"])


def _same_results(gk, gd, gn, rk, rd, rn, bitwise=True):
    assert np.array_equal(gn, rn)
    for b in range(len(gn)):
        n = gn[b]
        assert gk[b, :n].tolist() == rk[b, :n].tolist(), b
        if bitwise:
            assert _bit_equal(gd[b, :n], rd[b, :n]), b


@pytest.fixture(scope="module")
def ref():
    with open(os.path.join(GOLD, "reference_goldens.json")) as f:
        return json.load(f)


# ---------------------------------------------------------------- distances
def test_distance_kats(H, ref):
    for c in ref["distance"]:
        fn = H.CosineDistance if c["fn"] == "cosine" else H.EuclideanDistance
        d = fn(c["a"], c["b"])
        if "bits" in c:
            assert _bits(d) == int(c["bits"], 16), c["src"]
        else:
            assert abs(d - c["want"]) <= c["tol"], c["src"]


@pytest.mark.parametrize("dim", [1, 2, 3, 7, 16, 64, 100, 128, 255, 256, 500, 768, 1000, 1536, 2048, 2049, 3072,
                                 4096])
def test_distance_sweep_bitwise(H, O, dim):
    rng = np.random.default_rng(dim)
    X = rng.uniform(-1, 1, (300, dim)).astype(np.float32)
    X[7] = 0.0  # zero vector: cosine -> NaN like the reference
    q = rng.uniform(-1, 1, dim).astype(np.float32)
    for metric, fn in ((O.COSINE, H.CosineDistance), (O.EUCLIDEAN, H.EuclideanDistance)):
        got = fn.sweep(q, X)
        dev = np.array([O.distance(metric, O.ORDER_DEV, x, q) for x in X], np.float32)
        refd = np.array([O.distance(metric, O.ORDER_REF, x, q) for x in X], np.float32)
        assert _bit_equal(got, dev), (metric, dim)
        ok = ~np.isnan(refd)
        assert np.array_equal(np.isnan(got), np.isnan(refd))
        scale = np.maximum(1.0, np.abs(refd[ok])) if metric == O.EUCLIDEAN else 1.0
        assert np.all(np.abs(got[ok] - refd[ok]) <= TOL * scale)


# ---------------------------------------------------------------- goldens
def test_levels_match_oracle(H, O):
    g = H.Graph(M=16, Ml=0.25, EfSearch=20, Rng=42)
    want = _levels(O, O.COSINE, 16, 0.25, 20, 42, 500)
    assert np.array_equal(g.preview_levels(500), want)


def test_layer_node_search(H, ref):
    c = ref["layer_node_search"]
    g = H.Graph(M=6, Ml=0.5, EfSearch=c["ef"], Distance=H.EuclideanDistance)
    n = len(c["keys"])
    adj = -np.ones((1, n, 7), np.int32)
    for i, lst in c["adj"].items():
        adj[0, int(i), : len(lst)] = lst
    g.import_graph(np.array(c["keys"]), np.array(c["values"], np.float32), np.array([c["deg"]], np.int32), adj,
                   np.array([c["entry"]], np.int32))
    k, _, nres = g.search_arrays(np.array([c["query"]], np.float32), c["k"], mode=H.MODE_COMPAT)
    assert k[0, : nres[0]].tolist() == c["want_keys"]


def test_default_cosine(H, ref):
    c = ref["default_cosine"]
    g = H.Graph(M=c["M"], Ml=c["Ml"], EfSearch=c["EfSearch"], Distance=H.CosineDistance, Rng=1)
    g.Add(*[H.MakeNode(k, v) for k, v in zip(c["keys"], c["values"])])
    res = g.Search(c["query"], c["k"])
    assert [n.Key for n in res] == c["want_keys"]
    assert np.array_equal(res[0].Value, np.array(c["values"][0], np.float32))


@pytest.mark.parametrize("seed", range(6))
def test_add_search_1d(H, O, ref, seed):
    c = ref["add_search_1d"]
    n = c["n"]
    lv = _levels(O, O.EUCLIDEAN, c["M"], c["Ml"], c["EfSearch"], seed, n)
    o = O.Graph(metric=O.EUCLIDEAN, order=O.ORDER_DEV, M=c["M"], Ml=c["Ml"], EfSearch=c["EfSearch"])
    o.add(np.arange(n), np.arange(n, dtype=np.float32).reshape(-1, 1), lv)
    g = H.Graph(M=c["M"], Ml=c["Ml"], EfSearch=c["EfSearch"], Distance=H.EuclideanDistance)
    g.BatchAdd([H.MakeNode(i, [float(i)]) for i in range(n)], levels=lv)
    assert g.Topography() == o.topography()
    _same_graph(g.export(), o.export())
    res = [nd.Key for nd in g.Search(c["query"], c["k"])]
    rk, _, rn = o.search(c["query"], c["k"])
    assert res == rk[0, : rn[0]].tolist()
    assert len(res) == 4 and {64, 65} <= set(res)


# ---------------------------------------------------------------- compat build + search parity
def _fixture_cases():
    fx = np.load(os.path.join(GOLD, "oracle_fixtures.npz"))
    return fx, sorted({k.split("/")[0] for k in fx.files})


@pytest.mark.parametrize("name", ["c16_cos", "c8_l2", "c128_cos"])
def test_fixture_build_and_search(H, name):
    fx, _ = _fixture_cases()
    metric, M, ef = fx[f"{name}/cfg"].tolist()
    ml = float(fx[f"{name}/ml"][0])
    g = H.Graph(M=M, Ml=ml, EfSearch=ef, Distance=_metric_fn(H, metric))
    g.add_arrays(fx[f"{name}/keys"], fx[f"{name}/X"], levels=fx[f"{name}/levels"])
    ex = g.export()
    assert np.array_equal(ex["deg"], fx[f"{name}/deg"])
    L, N = ex["deg"].shape
    for l in range(L):
        for i in range(N):
            d = ex["deg"][l, i]
            if d > 0:
                assert set(ex["adj"][l, i, :d]) == set(fx[f"{name}/adj"][l, i, :d]), (l, i)
    for mname, mode in (("compat", H.MODE_COMPAT), ("beam", H.MODE_BEAM), ("exact", H.MODE_EXACT)):
        gk, gd, gn = g.search_arrays(fx[f"{name}/Q"], 10, mode=mode, ef=ef if mode != H.MODE_BEAM else 32)
        _same_results(gk, gd, gn, fx[f"{name}/{mname}_keys"], fx[f"{name}/{mname}_dist"], fx[f"{name}/{mname}_n"])


@pytest.mark.parametrize("n,d,metric,M,ml,ef", [
    (1500, 100, 0, 16, 0.25, 20),
    (1200, 768, 0, 16, 0.25, 20),
    (1500, 33, 1, 10, 0.3, 24),
    (800, 1536, 1, 12, 0.25, 16),
    (600, 3, 1, 6, 0.5, 20),
    (300, 3072, 0, 8, 0.25, 16),
    (250, 4096, 1, 6, 0.3, 16),
    # large M: the layer's eviction staging with 40-wide rows, and (M 60) a walk
    # whose staging area does not fit in LDS next to the rest (the plain path);
    # ef 64 also takes the LDS Go heaps instead of the register ones
    (700, 128, 1, 40, 0.25, 40),
    (500, 256, 0, 60, 0.25, 64),
])
def test_compat_build_parity(H, O, n, d, metric, M, ml, ef):
    rng = np.random.default_rng(n + d)
    X = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    if d > 4:
        X[n // 3] = 0.0  # zero vector: NaN distances follow the reference's comparisons
    Q = rng.uniform(-1, 1, (64, d)).astype(np.float32)
    keys = rng.permutation(5 * n)[:n].astype(np.int64) - n
    lv = _levels(O, metric, M, ml, ef, 77, n)
    o = O.Graph(metric=metric, order=O.ORDER_DEV, M=M, Ml=ml, EfSearch=ef)
    o.add(keys, X, lv)
    g = H.Graph(M=M, Ml=ml, EfSearch=ef, Distance=_metric_fn(H, metric))
    g.add_arrays(keys, X, levels=lv)
    _same_graph(g.export(), o.export())
    for mode in (H.MODE_COMPAT, H.MODE_BEAM, H.MODE_EXACT):
        for efq in ((ef, 50) if mode == H.MODE_COMPAT else (10, 64, 100, 200)):
            gk, gd, gn = g.search_arrays(Q, 10, mode=mode, ef=efq)
            rk, rd, rn = o.search(Q, 10, mode=mode, ef=efq)
            _same_results(gk, gd, gn, rk, rd, rn)
            if mode == H.MODE_EXACT:
                break
    # distances also within 1e-5 of the sequential fp32 restatement
    r = O.Graph(metric=metric, order=O.ORDER_REF, M=M, Ml=ml, EfSearch=ef)
    r.import_graph(**o.export())
    rk, rd, rn = r.search(Q, 10, mode=O.MODE_EXACT)
    gk, gd, gn = g.search_arrays(Q, 10, mode=H.MODE_EXACT)
    fin = np.isfinite(rd[:, 0])
    assert np.all(np.abs(gd[fin, 0] - rd[fin, 0]) <= TOL * np.maximum(1.0, np.abs(rd[fin, 0])))


@pytest.mark.parametrize("metric,d", [(0, 48), (1, 768)])
def test_compat_build_waves_identical(H, O, metric, d):
    """The compat insert scored by the walking wave alone or by 8 waves builds
    the same graph as the oracle."""
    rng = np.random.default_rng(d)
    n, M = 700, 10
    X = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    lv = _levels(O, metric, M, 0.3, 20, 5, n)
    o = O.Graph(metric=metric, order=O.ORDER_DEV, M=M, Ml=0.3, EfSearch=20)
    o.add(np.arange(n), X, lv)
    for waves in (1, 8):
        g = H.Graph(M=M, Ml=0.3, EfSearch=20, Distance=_metric_fn(H, metric), compat_waves=waves)
        g.add_arrays(np.arange(n), X, levels=lv)
        _same_graph(g.export(), o.export())
        g.close()


def test_entry_injection_and_incremental_adds(H, O):
    rng = np.random.default_rng(3)
    n, d = 900, 24
    X = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    Q = rng.uniform(-1, 1, (40, d)).astype(np.float32)
    lv = _levels(O, O.COSINE, 8, 0.25, 20, 5, n)
    o = O.Graph(metric=O.COSINE, order=O.ORDER_DEV, M=8, Ml=0.25, EfSearch=20)
    g = H.Graph(M=8, Ml=0.25, EfSearch=20)
    for a, b in ((0, 1), (1, 50), (50, 400), (400, n)):  # several Add calls grow the index
        o.add(np.arange(a, b), X[a:b], lv[a:b])
        g.add_arrays(np.arange(a, b), X[a:b], levels=lv[a:b])
    _same_graph(g.export(), o.export())
    top = len(o.topography()) - 1
    ex = o.export()
    members = [int(ex["keys"][i]) for i in range(n) if ex["deg"][top, i] != -2]
    for ek in members[:3]:
        gk, gd, gn = g.search_arrays(Q, 5, mode=H.MODE_COMPAT, entry_key=ek)
        rk, rd, rn = o.search(Q, 5, mode=O.MODE_COMPAT, entry_key=ek)
        _same_results(gk, gd, gn, rk, rd, rn)


# ---------------------------------------------------------------- API behaviour
def test_validation_and_errors(H):
    g = H.Graph(M=0, Ml=0.25, EfSearch=20)
    with pytest.raises(H.HnswError, match="M must be greater than 0, got 0"):
        g.Add(H.MakeNode(1, [1, 2, 3]))
    g = H.Graph(M=16, Ml=0.25, EfSearch=20)
    with pytest.raises(H.HnswError, match="k must be greater than 0, got 0"):
        g.Search([1, 2, 3], 0)
    assert g.Search([1, 2, 3], 3) == []  # empty graph: nil, nil (graph.go:554-556)
    g.Add(H.MakeNode(1, [1, 2, 3]))
    with pytest.raises(H.HnswError, match=r"embedding dimension mismatch: 3 != 2"):
        g.Add(H.MakeNode(2, [1, 2]))
    with pytest.raises(H.HnswError, match=r"embedding dimension mismatch: 3 != 2"):
        g.Search([1, 2], 1)
    with pytest.raises(H.HnswError, match=r"embedding dimension mismatch for query 1: 3 != 2"):
        g.BatchSearch([[1, 2, 3], [1, 2]], 1)
    assert g.Len() == 1 and g.Dims() == 3
    v, ok = g.Lookup(1)
    assert ok and v.tolist() == [1, 2, 3]
    assert g.Lookup(99) == (None, False)
    # a present key: BatchAdd's replacement (graph.go:1015-1024) ends the walk
    # with "node not added", or -- when the old node was also in a layer below
    # the replacing one's top -- the elevator names the deleted key and the
    # next layer's search fails (graph.go:1002-1010)
    with pytest.raises(H.HnswError, match="node not added|no nodes found in neighborhood search"):
        g.Add(H.MakeNode(1, [3, 2, 1]))


def test_batch_search_matches_search(H):
    rng = np.random.default_rng(8)
    g = H.Graph(M=8, Ml=0.25, EfSearch=20, Rng=4)
    X = rng.uniform(-1, 1, (300, 12)).astype(np.float32)
    g.BatchAdd([H.MakeNode(i, X[i]) for i in range(300)])
    Q = rng.uniform(-1, 1, (10, 12)).astype(np.float32)
    bs = g.BatchSearch(list(Q), 4)
    for q, r in zip(Q, bs):
        assert [n.Key for n in g.Search(q, 4)] == [n.Key for n in r]


def test_merge_topk_device(H):
    torch = pytest.importorskip("torch")
    S, B, k = 4, 257, 10
    rng = np.random.default_rng(1)
    dist = np.sort(rng.uniform(0, 1, (S, B, k)).astype(np.float32), axis=2)
    keys = rng.permutation(S * B * k).reshape(S, B, k).astype(np.int64)
    nn = rng.integers(0, k + 1, (S, B)).astype(np.int32)
    # compat lists carry NaN (zero rows under cosine) and signed zeros; exact ties across shards
    dist[0, :20, k - 3:] = np.nan
    dist[1, 20:40, k - 1] = np.nan
    dist[:, 40:60, 0] = -0.0
    dist[2, 60:80, 1] = 0.0
    dist[1, 80:100, :] = dist[0, 80:100, :]
    nn[:, :100] = k
    dev = torch.device("cuda:0")
    tk, td, tn = (torch.from_numpy(x).to(dev) for x in (keys, dist, nn))
    ok = torch.empty((B, k), dtype=torch.int64, device=dev)
    od = torch.empty((B, k), dtype=torch.float32, device=dev)
    on = torch.empty((B,), dtype=torch.int32, device=dev)
    H.merge_topk_device(tk.data_ptr(), td.data_ptr(), tn.data_ptr(), S, B, k, ok.data_ptr(), od.data_ptr(),
                        on.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ok, od, on = ok.cpu().numpy(), od.cpu().numpy(), on.cpu().numpy()
    from tests.test_distributed import merge_reference

    rk, rd, rn = (x.numpy() for x in merge_reference(keys, dist, nn, k))
    assert np.array_equal(on, rn)
    for b in range(B):
        assert ok[b, : on[b]].tolist() == rk[b, : rn[b]].tolist(), b
        assert np.array_equal(od[b, : on[b]], rd[b, : rn[b]], equal_nan=True), b


# ---------------------------------------------------------------- batched build
def _clustered(rng, n, d, nc=64, intrinsic=12, noise=0.05):
    C = rng.normal(size=(nc, intrinsic)).astype(np.float32)
    A = rng.normal(size=(intrinsic, d)).astype(np.float32) / np.sqrt(intrinsic)
    z = C[rng.integers(0, nc, n)] + 0.35 * rng.normal(size=(n, intrinsic)).astype(np.float32)
    x = z @ A + noise * rng.normal(size=(n, d)).astype(np.float32)
    return x.astype(np.float32)


@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("expand,upper_efc", [(1, 0), (2, 0), (3, 0), (4, 0), (4, 32)])
def test_batch_build_recall_and_exact_parity(H, O, metric, expand, upper_efc):
    """The batched insert at every expansion width (build_expand) and with a
    narrower candidate list above layer 0 (upper_efc): recall of the built graph,
    no dropped reverse-edge proposals, and the oracle's exact and beam searches
    on the same graph == the engine's."""
    rng = np.random.default_rng(11 + metric)
    n, d = 20000, 64
    X = _clustered(rng, n, d)
    Q = _clustered(rng, 200, d)
    g = H.Graph(M=16, Ml=0.25, EfSearch=64, Distance=_metric_fn(H, metric), Rng=9, build_mode=H.BUILD_BATCH,
                ef_construction=100, heuristic=2, build_expand=expand, upper_efc=upper_efc)
    assert g.get_option("upper_efc") == upper_efc
    g.add_arrays(np.arange(n), X)
    st = g.stats()
    assert st["dropped_proposals"] == 0
    ek, ed, en = g.search_arrays(Q, 10, mode=H.MODE_EXACT)

    def recall(ef):
        bk, bd, bn = g.search_arrays(Q, 10, mode=H.MODE_BEAM, ef=ef)
        return np.mean([len(set(bk[b, : bn[b]]) & set(ek[b, : en[b]])) / 10 for b in range(len(Q))]), (bk, bd, bn)

    # this off-centre clustered set is harder under cosine than under L2 (measured
    # 0.90 / 0.99 at ef=64 with efConstruction=100)
    r64, (bk, bd, bn) = recall(64)
    r128, _ = recall(128)
    assert r64 >= (0.85 if metric == 0 else 0.95), r64
    assert r128 >= 0.95 and r128 >= r64, (r64, r128)
    # same graph in the oracle: beam and exact identical
    o = O.Graph(metric=metric, order=O.ORDER_DEV, M=16, M0=32, Ml=0.25, EfSearch=64)
    o.import_graph(**g.export())
    rk, rd, rn = o.search(Q, 10, mode=O.MODE_EXACT)
    _same_results(ek, ed, en, rk, rd, rn)
    rk, rd, rn = o.search(Q, 10, mode=O.MODE_BEAM, ef=64)
    _same_results(bk, bd, bn, rk, rd, rn)


# ---------------------------------------------------------------- exact path: both scoring precisions
def _exact_inputs(rng, n, d, nq, metric):
    X = _clustered(rng, n, d)
    X[5] = X[17]                      # exact duplicates: ties broken by id
    X[6] = X[17]
    Q = _clustered(rng, nq, d)
    Q[1] = X[40]                      # a query equal to a stored row
    if metric == 0:
        X[9] = 0.0                    # zero row: NaN cosine, never returned
        Q[2] = 0.0                    # zero query: NaN everywhere, no results
    return X, Q


@pytest.mark.parametrize("precision", [0, 1, 2, 3])
@pytest.mark.parametrize("metric,d", [(0, 24), (1, 24), (0, 768), (1, 768), (0, 1536), (1, 4096)])
def test_exact_precision_parity(H, O, metric, d, precision):
    """Exact mode with f32-input MFMA scores (0), bf16x3 split scores (1) and
    fp16 2-product scores (2):
    after the canonical re-rank and the certificate (or its fallback) the
    output is the oracle's brute force bit for bit."""
    rng = np.random.default_rng(100 + d + metric)
    n = 3000 if d < 1536 else (1500 if d < 4096 else 600)
    X, Q = _exact_inputs(rng, n, d, 96, metric)
    g = H.Graph(M=8, Ml=0.25, EfSearch=32, Distance=_metric_fn(H, metric), Rng=3, build_mode=H.BUILD_BATCH,
                ef_construction=32)
    g.add_arrays(np.arange(n) * 7 + 3, X)
    g.set_option("exact_precision", precision)
    g.reset_stats()
    gk, gd, gn = g.search_arrays(Q, 10, mode=H.MODE_EXACT)
    o = O.Graph(metric=metric, order=O.ORDER_DEV, M=8, M0=16, Ml=0.25, EfSearch=32)
    o.import_graph(**g.export())
    rk, rd, rn = o.search(Q, 10, mode=O.MODE_EXACT)
    _same_results(gk, gd, gn, rk, rd, rn)
    if metric == 0:
        assert gn[2] == 0
    # clustered data leaves wide gaps at the preselection boundary: nearly every
    # query is certified without the fallback sweep
    assert g.stats()["exact_uncertified"] <= len(Q) // 4
    # a deleted row never comes back, in either precision
    g.Delete(int(gk[0, 0]))
    gk2, gd2, gn2 = g.search_arrays(Q[:1], 10, mode=H.MODE_EXACT)
    assert int(gk[0, 0]) not in gk2[0, : gn2[0]].tolist()
    g.close()


@pytest.mark.parametrize("k", [65, 200, 256])
def test_exact_large_k(H, O, k):
    """k up to 256 (multi-row preselection / re-rank lists), every precision."""
    rng = np.random.default_rng(k)
    n, d = 3000, 48
    X, Q = _exact_inputs(rng, n, d, 40, 0)
    g = H.Graph(M=8, Ml=0.25, EfSearch=32, Distance=H.CosineDistance, build_mode=H.BUILD_BATCH, ef_construction=32)
    g.add_arrays(np.arange(n), X)
    o = O.Graph(metric=0, order=O.ORDER_DEV, M=8, M0=16, Ml=0.25, EfSearch=32)
    o.import_graph(**g.export())
    rk, rd, rn = o.search(Q, k, mode=O.MODE_EXACT)
    for precision in (3, 2, 1, 0):
        g.set_option("exact_precision", precision)
        gk, gd, gn = g.search_arrays(Q, k, mode=H.MODE_EXACT)
        _same_results(gk, gd, gn, rk, rd, rn)
    with pytest.raises(H.HnswError, match="k <= 256"):
        g.search_arrays(Q[:1], 257, mode=H.MODE_EXACT)
    g.close()


@pytest.mark.parametrize("metric", [0, 1])
def test_exact_certificate_fallback(H, O, metric):
    """Preselection width kk = k leaves no margin, so the certificate fails for
    (nearly) every query; the canonical fallback sweep must still reproduce the
    oracle exactly -- across two score-workspace chunks (B > 4096)."""
    rng = np.random.default_rng(7 + metric)
    n, d, B = 400, 24, 4500
    X, _ = _exact_inputs(rng, n, d, 4, metric)
    Q = _clustered(rng, B, d)
    g = H.Graph(M=8, Ml=0.25, EfSearch=32, Distance=_metric_fn(H, metric), Rng=3, build_mode=H.BUILD_BATCH,
                ef_construction=32)
    g.add_arrays(np.arange(n), X)
    g.set_option("exact_kk", 10)
    for precision in (3, 2, 1, 0):
        g.set_option("exact_precision", precision)
        g.reset_stats()
        gk, gd, gn = g.search_arrays(Q, 10, mode=H.MODE_EXACT)
        assert g.stats()["exact_uncertified"] >= B // 2
        o = O.Graph(metric=metric, order=O.ORDER_DEV, M=8, M0=16, Ml=0.25, EfSearch=32)
        o.import_graph(**g.export())
        rk, rd, rn = o.search(Q, 10, mode=O.MODE_EXACT)
        _same_results(gk, gd, gn, rk, rd, rn)
    g.close()


@pytest.mark.parametrize("metric", [0, 1])
def test_exact_h16_outside_bound(H, O, metric):
    """fp16 2-product scores: rows outside the error bound's range (|x_i| up to
    1e15 or down to 1e-15, an infinite component) are always preselected and
    re-ranked canonically, queries outside it fail their certificate and are
    redone by the canonical sweep -- results still the oracle's brute force."""
    rng = np.random.default_rng(31 + metric)
    n, d = 2000, 64
    X, Q = _exact_inputs(rng, n, d, 48, metric)
    X[100] *= np.float32(1e15)
    X[101] *= np.float32(1e-15)
    X[102] *= np.float32(2.0 ** 39)                # inside the range, near its edges
    X[103] *= np.float32(2.0 ** -39)
    X[104, 3] = np.inf
    Q[5] *= np.float32(1e15)
    Q[6] *= np.float32(1e-15)
    Q[7] = X[101]                                 # finds the tiny row
    g = H.Graph(M=8, Ml=0.25, EfSearch=32, Distance=_metric_fn(H, metric), Rng=3, build_mode=H.BUILD_FLAT)
    g.add_arrays(np.arange(n), X)
    o = O.Graph(metric=metric, order=O.ORDER_DEV, M=8, M0=16, Ml=0.25, EfSearch=32)
    o.import_graph(**g.export())
    rk, rd, rn = o.search(Q, 10, mode=O.MODE_EXACT)
    # every precision; the huge query's L2 distances all tie in f32, so its top-k
    # is decided by ids alone (the preselection must admit rows tying its bound)
    for precision in (3, 2, 1, 0):
        g.set_option("exact_precision", precision)
        g.reset_stats()
        gk, gd, gn = g.search_arrays(Q, 10, mode=H.MODE_EXACT)
        if precision == 2:
            assert g.stats()["exact_uncertified"] >= 2     # the two out-of-range queries
        _same_results(gk, gd, gn, rk, rd, rn)
    g.close()


def test_dimension_limit(H):
    g = H.Graph(M=4, Ml=0.25, EfSearch=8)
    with pytest.raises(H.HnswError, match=r"dimension 4097 not supported \(1..4096\)"):
        g.add_arrays(np.arange(2), np.ones((2, 4097), np.float32))
    g.close()


# ---------------------------------------------------------------- Delete (graph.go:843-895)
def _live_connectivity(ex):
    out = []
    for l in range(ex["deg"].shape[0]):
        live = (ex["deg"][l] != -2) & (ex["dead"] == 0)
        if live.sum():
            out.append(float(np.maximum(ex["deg"][l][live], 0).sum()) / float(live.sum()))
    return out


def _search_parity(H, O, g, o, Q, k=10, efs=(20, 64)):
    for mode in (H.MODE_COMPAT, H.MODE_BEAM, H.MODE_EXACT):
        for ef in efs:
            gk, gd, gn = g.search_arrays(Q, k, mode=mode, ef=ef)
            rk, rd, rn = o.search(Q, k, mode=mode, ef=ef)
            try:
                _same_results(gk, gd, gn, rk, rd, rn)
            except AssertionError as e:
                raise AssertionError(f"mode {mode} ef {ef}: {e}") from None


@pytest.mark.parametrize("metric,M,ml,d", [(0, 8, 0.25, 24), (1, 6, 0.5, 3), (0, 16, 0.25, 768)])
def test_compat_delete_parity(H, O, metric, M, ml, d):
    """Delete/BatchDelete with the reference's isolate + replenish: identical
    graphs (rows, dead flags, entries), Len/Topography/Connectivity, and
    identical compat/beam/exact results afterwards; then more Adds."""
    rng = np.random.default_rng(21 + d)
    n = 700
    X = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    Q = rng.uniform(-1, 1, (48, d)).astype(np.float32)
    keys = np.arange(n, dtype=np.int64) * 3 - 500
    lv = _levels(O, metric, M, ml, 20, 31, n)
    o = O.Graph(metric=metric, order=O.ORDER_DEV, M=M, Ml=ml, EfSearch=20)
    g = H.Graph(M=M, Ml=ml, EfSearch=20, Distance=_metric_fn(H, metric))
    o.add(keys, X, lv)
    g.add_arrays(keys, X, levels=lv)
    gone = [int(x) for x in rng.choice(keys, 180, replace=False)]
    gone += gone[:3] + [123457]  # repeats and a missing key -> False
    ro = o.delete(gone)
    rg = g.BatchDelete(gone)
    assert ro == rg and rg[-4:] == [False] * 4
    ex = g.export()
    _same_graph(ex, o.export())
    assert g.Len() == len(o) == n - 180 and g.Topography() == o.topography()
    assert g.Connectivity() == _live_connectivity(ex)
    assert all(g.Lookup(k) == (None, False) for k in gone[:5])
    _search_parity(H, O, g, o, Q)
    # Adds after deletes (levels drawn from the live Len, graph.go:400).  A
    # deleted node reached through a dangling edge can become the elevator, and
    # the reference's Add then fails (graph.go:489-505); both sides must agree.
    lv2 = o.preview_levels(40)
    assert np.array_equal(lv2, g.preview_levels(40))
    _adds_agree(H, O, g, o, rng.uniform(-1, 1, (40, d)).astype(np.float32), 10**6, Q)


def _adds_agree(H, O, g, o, X2, key0, Q):
    """Add rows one at a time on both sides; identical graphs and results after
    each, or the same reference error on the same row (state after a failed
    Add is unspecified, so the walk stops there).  Returns rows added."""
    for i in range(len(X2)):
        lvl = o.preview_levels(1)
        oe = ge = None
        try:
            o.add([key0 + i], X2[i:i + 1], lvl)
        except O.OracleError as e:
            oe = str(e)
        try:
            g.add_arrays(np.array([key0 + i]), X2[i:i + 1], levels=lvl)
        except H.HnswError as e:
            ge = str(e)
        assert (oe is None) == (ge is None), (i, oe, ge)
        if oe is not None:
            assert "no nodes found in neighborhood search" in oe and "no nodes found in neighborhood search" in ge
            return i
        if i % 8 == 0 or i == len(X2) - 1:
            _same_graph(g.export(), o.export())
            _search_parity(H, O, g, o, Q, efs=(20,))
    return len(X2)


def test_compat_delete_top_layer_then_add(H, O):
    """Deleting every node of the top layers empties them; the next Add is
    taken by the emptied layers whatever its level (graph.go:485-488), and a
    later Add whose elevator is not in the layer below fails with the
    reference's "no nodes found in neighborhood search" (graph.go:500-505).
    Adds go one at a time so both sides hold identical graphs up to the first
    error."""
    rng = np.random.default_rng(9)
    n, d, M = 400, 8, 6
    X = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    lv = _levels(O, 0, M, 0.25, 20, 13, n)
    o = O.Graph(metric=0, order=O.ORDER_DEV, M=M, Ml=0.25, EfSearch=20)
    g = H.Graph(M=M, Ml=0.25, EfSearch=20)
    o.add(np.arange(n), X, lv)
    g.add_arrays(np.arange(n), X, levels=lv)
    top = int(lv.max())
    gone = [int(i) for i in np.flatnonzero(lv >= max(top - 1, 1))]
    assert o.delete(gone) == g.BatchDelete(gone) == [True] * len(gone)
    _same_graph(g.export(), o.export())
    Q = rng.uniform(-1, 1, (16, d)).astype(np.float32)
    _search_parity(H, O, g, o, Q, efs=(20,))
    added = _adds_agree(H, O, g, o, rng.uniform(-1, 1, (30, d)).astype(np.float32), n, Q)
    assert added >= 1 and o.topography()[top] >= 1  # the emptied top layer was taken by a new node


@pytest.mark.parametrize("metric", [0, 1])
def test_batch_delete_repair_parity(H, O, metric):
    """Batched-graph repair (k_delete_repair) == oracle repair_layer on the same
    graph; deleted keys never come back; recall holds; Adds continue."""
    rng = np.random.default_rng(40 + metric)
    n, d = 6000, 48
    X = _clustered(rng, n, d)
    Q = _clustered(rng, 200, d)
    g = H.Graph(M=12, Ml=0.25, EfSearch=64, Distance=_metric_fn(H, metric), Rng=3, build_mode=H.BUILD_BATCH,
                m0=24, ef_construction=64, heuristic=2, keep_pruned=1)
    g.add_arrays(np.arange(n), X)
    o = O.Graph(metric=metric, order=O.ORDER_DEV, M=12, M0=24, Ml=0.25, EfSearch=64)
    o.import_graph(**g.export())
    ex0 = g.export()
    top = ex0["deg"].shape[0] - 1
    gone = [int(ex0["keys"][ex0["entry"][top]])] + [int(x) for x in rng.permutation(n)[:900]]
    gone = list(dict.fromkeys(gone))
    assert g.BatchDelete(gone) == o.delete(gone, mode=1, heuristic=2, keep_pruned=1) == [True] * len(gone)
    ex = g.export()
    _same_graph(ex, o.export())
    dead = ex["dead"].astype(bool)
    for l in range(ex["deg"].shape[0]):
        rows = np.flatnonzero(~dead & (ex["deg"][l] > 0))
        for i in rows:
            assert not dead[ex["adj"][l, i, : ex["deg"][l, i]]].any()
    ek, ed, en = g.search_arrays(Q, 10, mode=H.MODE_EXACT)
    rk, rd, rn = o.search(Q, 10, mode=O.MODE_EXACT)
    _same_results(ek, ed, en, rk, rd, rn)
    bk, bd, bn = g.search_arrays(Q, 10, mode=H.MODE_BEAM, ef=64)
    rk, rd, rn = o.search(Q, 10, mode=O.MODE_BEAM, ef=64)
    _same_results(bk, bd, bn, rk, rd, rn)
    assert not set(bk[bn > 0].ravel().tolist()) & set(gone)
    r = np.mean([len(set(bk[b, : bn[b]]) & set(ek[b, : en[b]])) / 10 for b in range(len(Q))])
    assert r >= 0.85, r
    X2 = _clustered(rng, 1000, d)
    g.add_arrays(np.arange(n, n + 1000), X2)
    assert g.Len() == n - len(gone) + 1000
    ek, _, en = g.search_arrays(X2[:50], 1, mode=H.MODE_BEAM, ef=64)
    assert np.mean(ek[:, 0] == np.arange(n, n + 50)) >= 0.9


# ---------------------------------------------------------------- negatives (graph.go:1116-1537)
@pytest.mark.parametrize("metric,d", [(0, 24), (1, 768)])
def test_negatives_parity(H, O, metric, d):
    """Search-with-negatives on the GPU == the restatement: same candidates,
    bit-identical float32 scores, same order; every mode; 0..4 negatives."""
    rng = np.random.default_rng(70 + d)
    n = 900
    X = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    lv = _levels(O, metric, 12, 0.25, 20, 3, n)
    o = O.Graph(metric=metric, order=O.ORDER_DEV, M=12, Ml=0.25, EfSearch=20)
    g = H.Graph(M=12, Ml=0.25, EfSearch=20, Distance=_metric_fn(H, metric))
    o.add(np.arange(n), X, lv)
    g.add_arrays(np.arange(n), X, levels=lv)
    Q = rng.uniform(-1, 1, (30, d)).astype(np.float32)
    Q[3] = X[17]  # a query equal to a stored vector scores 2.0
    negs = [rng.uniform(-1, 1, (b % 5, d)).astype(np.float32) for b in range(30)]
    negs[5] = X[[40, 41]]  # candidates at distance 0 from a negative: the strong penalty
    for mode, ef in ((H.MODE_COMPAT, 0), (H.MODE_BEAM, 40), (H.MODE_EXACT, 0)):
        for k, w, flags in ((3, 0.5, 0), (7, 0.9, 1), (20, 0.0, 0)):
            gk, gs, gn = g.search_negatives_arrays(Q, negs, k, w, mode=mode, ef=ef, flags=flags)
            rk, rs, rn = o.search_negatives(Q, negs, k, w, mode=mode, ef=ef, flags=flags)
            _same_results(gk, gs, gn, rk, rs, rn)


def test_negatives_reference_cases(H):
    """negative_test.go:10-250 through the Python mirror of the Go API."""
    A = np.array([[1.0, 0.2, 0.1], [0.9, 0.3, 0.2], [0.8, 0.3, 0.3], [0.1, 1.0, 0.2], [0.2, 0.9, 0.3],
                  [0.3, 0.8, 0.3], [0.1, 0.2, 1.0], [0.2, 0.3, 0.9], [0.3, 0.3, 0.8]], np.float32)
    g = H.NewGraphWithConfig(16, 0.25, 20, H.CosineDistance)
    for i in range(9):
        g.Add(H.MakeNode(i + 1, A[i]))
    r = g.SearchWithNegative(A[0], A[1], 3, 0.5)
    assert len(r) == 3 and r[0].Key == 1
    r = g.SearchWithNegatives([0.4, 0.4, 0.4], [A[0], A[3]], 3, 0.7, flags=1)
    assert len(r) == 3 and any(7 <= n.Key <= 9 for n in r)
    assert [n.Key for n in g.SearchWithNegatives(A[0], [], 3, 0.5)] == [n.Key for n in g.Search(A[0], 3)]
    res = g.BatchSearchWithNegatives([A[0], A[3]], [[A[1]], [A[4]]], 3, 0.5)
    assert len(res) == 2 and res[0][0].Key == 1 and res[1][0].Key == 4
    res = g.BatchSearchWithNegatives([A[0], A[3]], [[], []], 3, 0.5)
    assert [[n.Key for n in x] for x in res] == [[n.Key for n in g.Search(q, 3)] for q in (A[0], A[3])]
    with pytest.raises(H.HnswError, match="negWeight must be between 0.0 and 1.0, got 1.500000"):
        g.SearchWithNegative(A[0], A[1], 3, 1.5)
    with pytest.raises(H.HnswError, match=r"negative embedding dimension mismatch: 3 != 2"):
        g.SearchWithNegative(A[0], [1, 2], 3, 0.5)
    with pytest.raises(H.HnswError, match=r"number of negative example sets \(1\) must match number of queries \(2\)"):
        g.BatchSearchWithNegatives([A[0], A[3]], [[A[1]]], 3, 0.5)
    assert [n.Key for n in g.ParallelSearch(A[0], 3)] == [n.Key for n in g.Search(A[0], 3)]
