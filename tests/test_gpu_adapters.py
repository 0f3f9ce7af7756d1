"""GPU: hnsw-extensions/hybrid adapters (hybrid/exact.go ExactIndex,
hybrid/adapter.go HNSWAdapter / ExactAdapter) over the engine.  ExactIndex is a
flat engine handle (no links) searched by the exact path; its answers must be
the oracle's canonical brute force, with the reference's replace-on-Add map
semantics."""
import numpy as np
import pytest

from tests.test_gpu_parity import _bit_equal, _clustered

pytestmark = pytest.mark.gpu


def _oracle_exact(O, metric, keys, X, Q, k):
    o = O.Graph(metric=metric, order=O.ORDER_DEV, M=8, Ml=0.25, EfSearch=20)
    o.add(np.asarray(keys, np.int64), X, np.zeros(len(keys), np.int32))
    return o.search(Q, k, mode=O.MODE_EXACT)


@pytest.mark.parametrize("metric", [0, 1])
def test_exact_index_matches_brute_force(H, O, metric):
    rng = np.random.default_rng(21 + metric)
    n, d, k = 2000, 24, 10
    X = _clustered(rng, n, d)
    Q = _clustered(rng, 40, d)
    keys = list(range(0, 3 * n, 3))
    idx = H.ExactIndex(H.CosineDistance if metric == 0 else H.EuclideanDistance)
    assert idx.Search(Q[0], k) == []  # empty index: no results, no error (exact.go:66-68)
    idx.BatchAdd(keys[:1500], X[:1500])
    for i in range(1500, n):
        idx.Add(keys[i], X[i])
    assert idx.Len() == n
    # replace-on-Add (a map assignment): 30 keys get new vectors in place, plus
    # 2 new keys in the same batch; Len grows by 2, the store by 2 rows only
    rows0 = idx._g.export()["keys"].shape[0]
    newv = _clustered(rng, 32, d)
    idx.BatchAdd(keys[100:130] + [1, 4], newv)
    assert idx.Len() == n + 2
    assert idx._g.export()["keys"].shape[0] == rows0 + 2
    X2 = np.concatenate([X, newv[30:]])
    X2[100:130] = newv[:30]
    keys2 = keys + [1, 4]
    order = list(range(n + 2))  # replaced rows keep their place (ties: insertion order)
    assert idx.BatchDelete([keys[5], keys[5], -7]) == [True, False, False]
    order.remove(5)
    # a batch that fails validation changes nothing
    with pytest.raises(H.HnswError, match="dimension mismatch"):
        idx.BatchAdd([keys[7], 99999], [np.ones(d, np.float32), np.ones(d + 1, np.float32)])
    assert idx.Len() == n + 1
    rk, rd, rn = _oracle_exact(O, metric, [keys2[i] for i in order], X2[order], Q, k)
    ks, od, on = idx.search_batch(Q, k)
    assert np.array_equal(on, rn)
    for b in range(len(Q)):
        assert ks[b] == rk[b, : rn[b]].tolist(), b
        assert _bit_equal(od[b, : on[b]], rd[b, : rn[b]]), b
    nodes = idx.Search(Q[3], k)
    assert [nd.Key for nd in nodes] == rk[3, : rn[3]].tolist()
    i0 = keys2.index(nodes[0].Key)
    assert np.array_equal(nodes[0].Value, X2[i0])
    with pytest.raises(H.HnswError) as e:
        idx.BatchAdd([1, 2], [X[0]])
    assert "number of keys (2) does not match number of vectors (1)" in str(e.value)
    with pytest.raises(H.HnswError):  # a flat handle has no graph to walk
        idx._g.search_arrays(Q[:1], k, mode=H.MODE_BEAM)
    idx.Close()


def test_adapters(H, O):
    rng = np.random.default_rng(33)
    n, d = 800, 16
    X = _clustered(rng, n, d)
    Q = _clustered(rng, 10, d)
    g = H.Graph(M=8, Ml=0.25, EfSearch=32, Distance=H.CosineDistance, build_mode=H.BUILD_BATCH, ef_construction=64)
    a = H.HNSWAdapter(g, H.CosineDistance, mode=H.MODE_BEAM)
    errs = a.BatchAdd([f"k{i}" for i in range(n)], X)
    assert errs == [None] * n and a.Len() == n
    assert "does not match" in str(a.BatchAdd(["x"], [])[0])
    for q in Q:
        ks, ds = a.Search(q, 5)
        assert len(ks) == 5 and all(isinstance(x, str) for x in ks)
        for key, dist in zip(ks, ds):
            v, ok = g.Lookup(key)
            # the reference recomputes a.distance(query, node.Value) (adapter.go:62-64): same canonical value
            assert ok and np.float32(dist) == H.CosineDistance(q, v)
    assert a.Delete("k3") and a.BatchDelete(["k4", "nope"]) == [True, False] and a.Len() == n - 2
    with pytest.raises(H.HnswError, match="flat"):  # in-place replacement is for vector stores only
        g.Replace([H.Node("k5", X[0])])
    e = H.ExactAdapter(H.ExactIndex(H.CosineDistance))
    assert e.Search(Q[0], 3) == ([], [])
    assert e.BatchAdd(list(range(n)), X) == [None] * n
    ks, ds = e.Search(Q[0], 5)
    idx_nodes = e.index.Search(Q[0], 5)
    assert ks == [nd.Key for nd in idx_nodes] and ds == sorted(ds)
    assert e.Delete(ks[0]) and e.Search(Q[0], 5)[0][0] == ks[1]
    e.Close()
    g.close()
