"""GPU parity of BatchAdd on keys that are already present (graph.go:1015-1024,
1035-1037) and of keys that come back after a Delete (graph.go:50 map
assignment): the HIP engine against the oracle on identical inputs --
identical rows, adjacency, entries, dead flags, Len/Topography/Connectivity,
the same errors at the same inserts, and identical compat / beam / exact
results afterwards."""
import numpy as np
import pytest

from tests.test_gpu_parity import _live_connectivity, _metric_fn, _same_graph, _search_parity

pytestmark = pytest.mark.gpu


def _agree(H, O, g, o, Q, efs=(20,)):
    ex = g.export()
    _same_graph(ex, o.export())
    assert g.Len() == len(o) and g.Topography() == o.topography()
    assert g.Connectivity() == _live_connectivity(ex)
    _search_parity(H, O, g, o, Q, efs=efs)


def _both_add(H, O, g, o, keys, X, levels=None):
    """The same BatchAdd on both sides -> the common error text (None: no error)."""
    oe = ge = None
    try:
        o.add(keys, X, levels)
    except O.OracleError as e:
        oe = str(e)
    try:
        g.add_arrays(np.asarray(keys, np.int64), X, levels=levels)
    except H.HnswError as e:
        ge = str(e)
    assert oe == ge, (oe, ge)
    return oe


def _walk_len(live, keys):
    """inserts BatchAdd reaches: through the first key present (or repeated)"""
    seen = set()
    for i, k in enumerate(keys):
        if k in live or k in seen:
            return i + 1
        seen.add(k)
    return len(keys)


@pytest.mark.parametrize("metric,M,ml,d,seeded", [(0, 8, 0.25, 24, False), (1, 6, 0.5, 5, True),
                                                  (0, 10, 0.3, 48, True)])
def test_readd_live_keys(H, O, metric, M, ml, d, seeded):
    """A stream of batches where 20 % of the keys are live ones (some with
    their old vector, so the old node is the nearest -- the elevator then names
    the replaced key and the reference's walk fails one layer down): each call
    inserts up to the first present key, replaces it and stops with "node not
    added"; the caller goes on with the rest."""
    rng = np.random.default_rng(100 + d)
    n = 500
    X = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    keys = (rng.permutation(4 * n)[:n] * 7 - 900).astype(np.int64)
    Q = rng.uniform(-1, 1, (32, d)).astype(np.float32)
    seed = 4242
    o = O.Graph(metric=metric, order=O.ORDER_DEV, M=M, Ml=ml, EfSearch=20, seed=seed)
    g = H.Graph(M=M, Ml=ml, EfSearch=20, Distance=_metric_fn(H, metric), Rng=seed)
    lv0 = None if seeded else o.preview_levels(n)
    assert _both_add(H, O, g, o, keys, X, lv0) is None
    _agree(H, O, g, o, Q)
    vec = {int(k): X[i] for i, k in enumerate(keys)}
    fresh = 10**6
    errors = {}
    for step in range(30):
        cnt = int(rng.integers(1, 9))
        ks, vs = [], []
        for _ in range(cnt):
            r = rng.random()
            if r < 0.2:
                k = int(rng.choice(list(vec)))
                ks.append(k)
                vs.append(vec[k] if rng.random() < 0.3 else rng.uniform(-1, 1, d).astype(np.float32))
            else:
                ks.append(fresh)
                fresh += 1
                vs.append(rng.uniform(-1, 1, d).astype(np.float32))
        if step % 7 == 3 and ks:  # a key repeated inside one batch
            ks.append(ks[0])
            vs.append(rng.uniform(-1, 1, d).astype(np.float32))
        V = np.stack(vs)
        w = _walk_len(vec, ks)
        lv = None if seeded else np.array([o.random_level() for _ in range(w)], np.int32)
        if lv is not None:
            lv = np.concatenate([lv, np.zeros(len(ks) - w, np.int32)])
        err = _both_add(H, O, g, o, ks, V, lv)
        errors[err] = errors.get(err, 0) + 1
        # the model of live keys (layer 0) from the oracle: a walk goes on past a key
        # whose nodes sat only in upper layers, and stops part way on a failure
        ex = o.export()
        live = ex["dead"] == 0
        vec = {int(k): ex["vecs"][i] for i, k in enumerate(ex["keys"]) if live[i] and ex["deg"][0, i] != -2}
        _agree(H, O, g, o, Q)
        if seeded:
            assert np.array_equal(g.preview_levels(8), o.preview_levels(8))
    assert errors.get("node not added", 0) >= 3, errors
    for k in list(vec)[:20]:  # Lookup: the replacing value
        v, ok = g.Lookup(k)
        assert ok and np.array_equal(v, vec[k])


def test_duplicate_inside_one_batch(H, O):
    """[a, b, a]: a and b are inserted, the second a replaces the first."""
    rng = np.random.default_rng(5)
    d, n = 16, 200
    X = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    Q = rng.uniform(-1, 1, (16, d)).astype(np.float32)
    o = O.Graph(metric=O.COSINE, order=O.ORDER_DEV, M=8, Ml=0.25, EfSearch=20, seed=9)
    g = H.Graph(M=8, Ml=0.25, EfSearch=20, Rng=9)
    assert _both_add(H, O, g, o, np.arange(n), X) is None
    V = rng.uniform(-1, 1, (4, d)).astype(np.float32)
    assert _both_add(H, O, g, o, [5000, 5001, 5000, 5002], V) == "node not added"
    _agree(H, O, g, o, Q)
    assert len(o) == n + 2  # 5002 never ran
    v, ok = g.Lookup(5000)
    assert ok and np.array_equal(v, V[2])
    assert g.Lookup(5002) == (None, False)


@pytest.mark.parametrize("metric", [0, 1])
def test_delete_then_readd(H, O, metric):
    """Delete 30 % of the keys, then add the same keys with new vectors at
    768-d: nodes still holding a dangling entry of a key get it overwritten
    when the new node links to them (graph.go:50), searches visit a key once."""
    rng = np.random.default_rng(77 + metric)
    n, d, M = 400, 768, 16
    X = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    Q = rng.uniform(-1, 1, (24, d)).astype(np.float32)
    keys = np.arange(n, dtype=np.int64) * 2 + 1
    o = O.Graph(metric=metric, order=O.ORDER_DEV, M=M, Ml=0.25, EfSearch=20, seed=31)
    g = H.Graph(M=M, Ml=0.25, EfSearch=20, Distance=_metric_fn(H, metric), Rng=31)
    assert _both_add(H, O, g, o, keys, X) is None
    gone = [int(k) for k in rng.choice(keys, 120, replace=False)]
    assert o.delete(gone) == g.BatchDelete(gone)
    _agree(H, O, g, o, Q, efs=(20, 64))
    back = list(gone)
    rng.shuffle(back)
    errs = tries = 0
    while back and tries < 40:
        tries += 1
        ks, back = back[:10], back[10:]
        V = rng.uniform(-1, 1, (len(ks), d)).astype(np.float32)
        err = _both_add(H, O, g, o, ks, V)
        assert err in (None, "no nodes found in neighborhood search", "node not added"), err
        if err is not None:  # the walk stopped part way: the keys it did not add go again
            errs += 1
            ex = o.export()
            in0 = {int(k) for i, k in enumerate(ex["keys"]) if ex["dead"][i] == 0 and ex["deg"][0, i] != -2}
            back += [k for k in ks if k not in in0]
        _agree(H, O, g, o, Q)
    assert g.Len() == len(o) and errs > 0
    assert np.array_equal(g.preview_levels(8), o.preview_levels(8))


def test_host_rng_draws_follow_the_walk(H, O):
    """With a host Rng, a BatchAdd that stops at a replacement draws levels only
    for the inserts it reached (graph.go:962): the next Add's levels continue
    the same stream, so the graph equals the oracle's (same seed)."""
    rng = np.random.default_rng(8)
    d, n = 12, 300
    X = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    Q = rng.uniform(-1, 1, (16, d)).astype(np.float32)
    o = O.Graph(metric=O.COSINE, order=O.ORDER_DEV, M=6, Ml=0.25, EfSearch=20, seed=77)
    g = H.Graph(M=6, Ml=0.25, EfSearch=20, Rng=H.SplitMix64Rand(77))
    o.add(np.arange(n), X)
    g.BatchAdd([H.Node(i, X[i]) for i in range(n)])
    _agree(H, O, g, o, Q)
    for step in range(6):
        ks = [10_000 + 10 * step + j for j in range(5)] + [int(rng.integers(0, n))] + [20_000 + step]
        V = rng.uniform(-1, 1, (len(ks), d)).astype(np.float32)
        with pytest.raises(O.OracleError, match="node not added"):
            o.add(ks, V)
        with pytest.raises(H.HnswError, match="node not added"):
            g.BatchAdd([H.Node(k, V[i]) for i, k in enumerate(ks)])
        _agree(H, O, g, o, Q)
    # a dimension mismatch part way: the nodes before it stay added (graph.go:955-960)
    with pytest.raises(H.HnswError, match="embedding dimension mismatch: 12 != 3"):
        g.BatchAdd([H.Node(30_000, X[0]), H.Node(30_001, X[1]), H.Node(30_002, X[2][:3])])
    o.add([30_000, 30_001], X[:2])
    _agree(H, O, g, o, Q)


class _PlainRng:
    """a host Rng with Float64() only (Go's *rand.Rand: no way to rewind it)"""

    def __init__(self, seed, H):
        self._r = H.SplitMix64Rand(seed)

    def Float64(self):
        return self._r.Float64()


@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("kind", ["rewind", "plain"])
def test_host_rng_walk_after_deletes(H, O, metric, kind, monkeypatch):
    """A host Rng (Go's *rand.Rand stand-in) on an index with deleted rows,
    where inserts can fail part way (graph.go:1009).  A Rng that can be rewound
    (SplitMix64Rand: getstate / setstate) keeps each BatchAdd ONE mhnsw_add
    call -- after a failure the engine reports how many inserts the walk
    reached (mhnsw_add_reached) and the host restores its Rng and redraws
    exactly those inserts' draws (graph.go:962); one that cannot goes one
    insert per call.  Either way the next Add's levels continue the
    reference's stream, and no draw is held back from the Rng: every step
    equals the oracle drawing from the same seed itself."""
    rng = np.random.default_rng(177 + metric)
    n, d, M = 400, 32, 8
    X = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    Q = rng.uniform(-1, 1, (24, d)).astype(np.float32)
    keys = np.arange(n, dtype=np.int64) * 2 + 1
    o = O.Graph(metric=metric, order=O.ORDER_DEV, M=M, Ml=0.25, EfSearch=20, seed=31)
    g = H.Graph(M=M, Ml=0.25, EfSearch=20, Distance=_metric_fn(H, metric),
                Rng=H.SplitMix64Rand(31) if kind == "rewind" else _PlainRng(31, H))
    assert _both_add(H, O, g, o, keys, X) is None
    gone = [int(k) for k in rng.choice(keys, 45, replace=False)]
    assert o.delete(gone) == g.BatchDelete(gone)
    _agree(H, O, g, o, Q)
    lib = H.load()
    real = lib.mhnsw_add
    calls = [0]

    def counted(*args):
        calls[0] += 1
        return real(*args)

    monkeypatch.setattr(lib, "mhnsw_add", counted)
    back = list(gone)
    rng.shuffle(back)
    errs = adds = 0
    while back and adds < 60:
        adds += 1
        ks, back = back[:12], back[12:]
        V = rng.uniform(-1, 1, (len(ks), d)).astype(np.float32)
        err = _both_add(H, O, g, o, ks, V)
        assert err in (None, "no nodes found in neighborhood search"), err
        if err is not None:
            errs += 1
            ex = o.export()
            in0 = {int(k) for i, k in enumerate(ex["keys"]) if ex["dead"][i] == 0 and ex["deg"][0, i] != -2}
            back += [k for k in ks if k not in in0 and k not in back]
        _agree(H, O, g, o, Q)
    print({"adds": adds, "failed": errs, "mhnsw_add_calls": calls[0]})
    assert 0 < errs < adds, (errs, adds)
    if kind == "rewind":
        assert calls[0] <= adds, (calls[0], adds)
    else:
        assert calls[0] > adds, (calls[0], adds)
    assert g.Len() == len(o)


def test_add_plan_and_contains(H):
    g = H.Graph(M=4, Ml=0.25, EfSearch=10, Rng=1)
    X = np.random.default_rng(1).uniform(-1, 1, (10, 8)).astype(np.float32)
    g.add_arrays(np.arange(10), X)
    assert g.contains([3, 10, 9, -1]).tolist() == [True, False, True, False]
    import ctypes as C
    lib = H.load()
    for ks, want in (([20, 21, 3, 22], 3), ([20, 21, 20, 5], 3), ([20, 21], 2), ([4], 1)):
        a = np.array(ks, np.int64)
        w, one = C.c_int64(), C.c_int()
        assert lib.mhnsw_add_plan(g._h, a.ctypes.data_as(C.POINTER(C.c_int64)), len(a), C.byref(w), C.byref(one)) == 0
        assert (w.value, one.value) == (want, 0)
    g.BatchDelete([0])
    a = np.array([99], np.int64)
    w, one = C.c_int64(), C.c_int()
    lib.mhnsw_add_plan(g._h, a.ctypes.data_as(C.POINTER(C.c_int64)), 1, C.byref(w), C.byref(one))
    assert one.value == 1  # a dangling elevator can now fail an insert: one at a time


def test_batch_mode_rejects_present_keys(H):
    g = H.Graph(M=8, Ml=0.25, EfSearch=20, Rng=1, build_mode=H.BUILD_BATCH)
    X = np.random.default_rng(2).uniform(-1, 1, (50, 8)).astype(np.float32)
    g.add_arrays(np.arange(50), X)
    with pytest.raises(H.HnswError, match="compat build mode"):
        g.add_arrays(np.array([3]), X[:1])
    assert g.Len() == 50


@pytest.mark.parametrize("compat,dup", [(True, False), (True, True), (False, False)])
def test_add_capacity_failure_leaves_index_unchanged(H, O, compat, dup):
    """An Add that fails on the host after its bookkeeping began (here the row
    capacity limit, `max_rows`; in practice a device allocation) leaves the
    index as it was: Len, layers, key maps and the engine's Rng.  The same Add
    afterwards -- and every search -- then agrees with a twin index that never
    saw the failure (the compat twin is also the oracle's graph: same levels,
    same walk).  With `dup` the failing batch ends in a present key, so the
    failure comes after the replacement's bookkeeping."""
    rng = np.random.default_rng(31 + compat + 2 * dup)
    n, m, d = 400, 40, 24
    X = rng.uniform(-1, 1, (n + m, d)).astype(np.float32)
    keys = np.arange(n + m, dtype=np.int64) * 3 + 7
    Q = rng.uniform(-1, 1, (24, d)).astype(np.float32)
    kw = {} if compat else dict(build_mode=H.BUILD_BATCH, m0=16, ef_construction=40, heuristic=2)
    a = H.Graph(M=8, Ml=0.25, EfSearch=20, Distance=H.CosineDistance, Rng=9, **kw)
    b = H.Graph(M=8, Ml=0.25, EfSearch=20, Distance=H.CosineDistance, Rng=9, **kw)
    bk, bx = keys[n:], X[n:]
    if dup:
        bk, bx = np.concatenate([bk, keys[:1]]), np.concatenate([bx, X[:1]])
    for g in (a, b):
        g.add_arrays(keys[:n], X[:n])
    a.set_option("max_rows", n + 10)
    with pytest.raises(H.HnswError) as e:
        a.add_arrays(bk, bx)
    assert "max_rows" in str(e.value)
    assert a.Len() == n and a.Topography() == b.Topography()
    a.set_option("max_rows", 0)
    errs = []
    for g in (a, b):
        try:
            g.add_arrays(bk, bx)
            errs.append(None)
        except H.HnswError as e2:
            errs.append(str(e2))
    assert errs[0] == errs[1] and errs[0] == ("node not added" if dup else None), errs
    ea, eb = a.export(), b.export()
    for name in ("keys", "vecs", "deg", "adj", "entry", "dead"):
        assert np.array_equal(np.asarray(ea[name]), np.asarray(eb[name])), name
    modes = (H.MODE_COMPAT, H.MODE_BEAM, H.MODE_EXACT) if compat else (H.MODE_BEAM, H.MODE_EXACT)
    for mode in modes:
        ra, rb = a.search_arrays(Q, 10, mode=mode), b.search_arrays(Q, 10, mode=mode)
        for x, y in zip(ra, rb):
            assert np.array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8)), mode
    if compat:  # and the twin is the oracle's graph
        o = O.Graph(metric=O.COSINE, order=O.ORDER_DEV, M=8, Ml=0.25, EfSearch=20)
        o.import_graph(**eb)
        _search_parity(H, O, b, o, Q)
    a.close()
    b.close()


def _partial_keys(o):
    """keys with a live node outside layer 0 (left by a failed insert), and their layers"""
    ex = o.export()
    out = {}
    for i, k in enumerate(ex["keys"]):
        if ex["dead"][i] == 0 and ex["deg"][0, i] == -2:
            layers = [l for l in range(ex["deg"].shape[0]) if ex["deg"][l, i] != -2]
            if layers:  # (a failed insert's row that reached no layer is no node)
                out[int(k)] = layers
    return out


@pytest.mark.parametrize("metric", [0, 1])
def test_partial_nodes_resolved_per_layer(H, O, metric):
    """A failed insert (graph.go:1009) leaves its node in the layers above the
    failing one.  The reference's layer maps are keyed by K, so:
      * a later insert of that key at or above one of those layers sweeps the
        old node (graph.go:1015-1024) and -- layer 0 never held it -- Len()
        grows: no "node not added", BatchAdd goes on with the next nodes;
      * an insert of that key below all of them adds a second live node; each
        layer's map resolves the key to the node it holds (the elevator,
        graph.go:997-1003, 574), Lookup to the layer-0 one, Delete removes both.
    Ops are driven identically on the engine and the oracle; every step agrees
    (rows, adjacency, errors, compat / beam / exact results)."""
    rng = np.random.default_rng(921)  # (a stream where a swept key's walk goes on, both metrics)
    n, d, M = 600, 8, 6
    X = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    keys = np.arange(n, dtype=np.int64) * 3 + 1
    o = O.Graph(metric=metric, order=O.ORDER_DEV, M=M, Ml=0.5, EfSearch=16, seed=55)
    g = H.Graph(M=M, Ml=0.5, EfSearch=16, Distance=_metric_fn(H, metric), Rng=55)
    assert _both_add(H, O, g, o, keys, X) is None
    Q = rng.uniform(-1, 1, (24, d)).astype(np.float32)
    # delete most of the graph, then add keys back at high levels: elevators through
    # deleted nodes fail inserts part way
    gone = [int(k) for k in rng.choice(keys, int(0.6 * n), replace=False)]
    assert o.delete(gone) == g.BatchDelete(gone)
    _agree(H, O, g, o, Q)
    fresh = 10**6
    seen = {"continue": 0, "second": 0, "went_on": 0}
    for step in range(60):
        part = _partial_keys(o)
        ks, lv = [], []
        cont_step = False
        if part and step % 2 == 0:
            k = int(rng.choice(list(part)))
            top = max(part[k])
            if rng.random() < 0.5:  # at or above one of its layers: swept, the walk goes on
                ks.append(k)
                lv.append(int(rng.integers(min(part[k]), top + 2)))
                seen["continue"] += 1
                cont_step = True
            elif min(part[k]) > 0:  # below all of them: a second live node
                ks.append(k)
                lv.append(int(rng.integers(0, min(part[k]))))
                seen["second"] += 1
        for _ in range(int(rng.integers(1, 5))):
            r = rng.random()
            ks.append(int(rng.choice(gone)) if r < 0.5 else fresh)
            fresh += r >= 0.5
            lv.append(int(rng.integers(0, 5)))
        V = rng.uniform(-1, 1, (len(ks), d)).astype(np.float32)
        err = _both_add(H, O, g, o, ks, V, np.array(lv, np.int32))
        assert err in (None, "no nodes found in neighborhood search", "node not added"), err
        _agree(H, O, g, o, Q, efs=(16, 40))
        if cont_step and len(ks) > 1:  # the walk went on past the swept key (whatever stopped it later)
            import ctypes as C
            reached = C.c_int64()
            assert H.load().mhnsw_add_reached(g._h, C.byref(reached)) == 0
            if reached.value >= 2:
                seen["went_on"] += 1
            if err is None:
                assert reached.value == len(ks) and all(g.Lookup(k)[1] for k in ks[1:]), ks
        for k in ks:  # Lookup = layers[0].nodes[key]
            gv, gok = g.Lookup(k)
            ex = o.export()
            rows = [i for i, kk in enumerate(ex["keys"]) if kk == k and ex["dead"][i] == 0 and ex["deg"][0, i] != -2]
            assert gok == bool(rows), k
            if rows:
                assert np.array_equal(gv, ex["vecs"][rows[0]]), k
        if step % 10 == 9:  # Delete removes every node of a key
            dk = list(_partial_keys(o))[:3] + [int(rng.choice(keys))]
            assert o.delete(dk) == g.BatchDelete(dk)
            _agree(H, O, g, o, Q)
    print(seen)
    assert seen["continue"] > 0 and seen["second"] > 0 and seen["went_on"] > 0, seen
