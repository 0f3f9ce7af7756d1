"""GPU: Go key types beyond `int` (Graph[K cmp.Ordered], graph.go:305).  The
engine compares keys only by order, so string keys travel as order labels
(mhnsw_strkeys_encode) and float keys as their IEEE total-order image.  A
graph keyed by strings / floats must behave exactly like the same graph keyed
by each key's rank: the oracle (keyed by ranks) is the checker."""
import numpy as np
import pytest

from tests import go_format as F
from tests.test_gpu_parity import _levels, _same_results

pytestmark = pytest.mark.gpu


def _words(rng, n):
    alpha = np.array(list("abcdefghijklmnopqrstuvwxyz"))
    out = set()
    while len(out) < n:
        out.add("".join(rng.choice(alpha, rng.integers(1, 7))))
    return list(out)


def _ranked(keys):
    order = {k: i for i, k in enumerate(sorted(keys))}
    return np.array([order[k] for k in keys], np.int64), sorted(keys)


def _check_against_rank_oracle(H, O, g, keys, X, lv, Q, metric, M):
    """oracle keyed by ranks, same insertion order and levels"""
    ranks, srt = _ranked(keys)
    o = O.Graph(metric=metric, order=O.ORDER_DEV, M=M, Ml=0.25, EfSearch=20)
    o.add(ranks, X, lv)
    for mode in (H.MODE_COMPAT, H.MODE_BEAM, H.MODE_EXACT):
        gk, gd, gn = g.search_arrays(Q, 10, mode=mode, ef=32)
        rk, rd, rn = o.search(Q, 10, mode=mode, ef=32)
        assert np.array_equal(gn, rn)
        for b in range(len(Q)):
            got = g.decode_keys(gk[b, : gn[b]])
            assert got == [srt[r] for r in rk[b, : rn[b]]], (mode, b)
        _same_results(np.zeros_like(gk), gd, gn, np.zeros_like(rk), rd, rn)  # distances bit-identical
    return o


@pytest.mark.parametrize("metric", [0, 1])
def test_string_keys_match_rank_keys(H, O, metric):
    rng = np.random.default_rng(5 + metric)
    n, d, M = 700, 16, 8
    keys = _words(rng, n)
    X = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    lv = _levels(O, metric, M, 0.25, 20, 3, n)
    g = H.Graph(M=M, Ml=0.25, EfSearch=20, Distance=H.CosineDistance if metric == 0 else H.EuclideanDistance)
    # a bulk batch, then batches small enough for incremental labels, then singles
    cuts = [0, 400, 520, 600, 650] + list(range(651, n + 1))
    for a, b in zip(cuts[:-1], cuts[1:]):
        g.BatchAdd([H.MakeNode(keys[i], X[i]) for i in range(a, b)], levels=lv[a:b])
    assert g.get_option("strkeys") == n
    Q = rng.uniform(-1, 1, (48, d)).astype(np.float32)
    _check_against_rank_oracle(H, O, g, keys, X, lv, Q, metric, M)
    # Node API: keys and the caller's values come back
    res = g.Search(X[123], 3, mode=H.MODE_EXACT)
    assert res[0].Key == keys[123] and np.array_equal(res[0].Value, X[123])
    v, ok = g.Lookup(keys[77])
    assert ok and np.array_equal(v, X[77])
    assert g.Lookup("not-a-key")[1] is False
    # Delete by string key
    assert g.Delete(keys[123]) and not g.Delete(keys[123]) and not g.Delete("not-a-key")
    bk, _, bn = g.search_arrays(X[123:124], 10, mode=H.MODE_BEAM, ef=32)
    assert keys[123] not in g.decode_keys(bk[0, : bn[0]])
    g.close()


def test_string_label_respacing(H, O):
    """Keys inserted one by one into the same gap exhaust the midpoints; the
    engine re-spaces every label and rewrites the stored keys -- results stay
    identical to the rank-keyed oracle."""
    rng = np.random.default_rng(9)
    base = [f"b{i:02d}" for i in range(100)]
    squeeze = ["b50" + "0" * i for i in range(1, 81)]  # b500 < b5000 < ... < b51
    keys = base + squeeze
    n, d, M = len(keys), 12, 6
    X = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    lv = _levels(O, 0, M, 0.25, 20, 4, n)
    g = H.Graph(M=M, Ml=0.25, EfSearch=20, Distance=H.CosineDistance)
    g.BatchAdd([H.MakeNode(keys[i], X[i]) for i in range(100)], levels=lv[:100])
    r0 = g.get_option("strkey_relabels")
    for i in range(100, n):
        g.BatchAdd([H.MakeNode(keys[i], X[i])], levels=lv[i:i + 1])
    assert g.get_option("strkey_relabels") > r0
    Q = rng.uniform(-1, 1, (32, d)).astype(np.float32)
    _check_against_rank_oracle(H, O, g, keys, X, lv, Q, 0, M)
    g.close()


def test_string_keys_export_import(H, O):
    """encode.go with K = string: the engine's bytes == the restatement's (with
    deletions), and an import of a file reproduces the graph (same results,
    same strings, same bytes on re-export)."""
    rng = np.random.default_rng(13)
    n, d, M = 300, 8, 6
    keys = _words(rng, n)
    X = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    lv = _levels(O, 0, M, 0.25, 20, 5, n)

    def build():
        g = H.Graph(M=M, Ml=0.25, EfSearch=20, Distance=H.CosineDistance)
        g.BatchAdd([H.MakeNode(keys[i], X[i]) for i in range(n)], levels=lv)
        return g

    g = build()
    g.BatchDelete(keys[:20])
    ex = g.export()
    lab2s = dict(zip(ex["keys"].tolist(), g.decode_keys(ex["keys"])))
    buf = g.export_bytes()
    assert buf == F.encode_export(ex, g.M, g.Ml, g.EfSearch, "cosine", F.KEY_STRING, keymap=lab2s.get)
    dec = F.decode(buf, F.KEY_STRING)
    assert {k for k, _, _ in dec["layers"][0]} == set(keys[20:])
    g.close()

    g = build()
    buf = g.export_bytes()
    h = H.Graph()
    h.import_bytes(buf, H.KEY_STRING)
    assert h.Len() == n and h.get_option("strkeys") == n
    Q = rng.uniform(-1, 1, (24, d)).astype(np.float32)
    for mode in (H.MODE_COMPAT, H.MODE_BEAM, H.MODE_EXACT):
        a = g.search_arrays(Q, 5, mode=mode)
        b = h.search_arrays(Q, 5, mode=mode)
        assert np.array_equal(a[2], b[2])
        assert np.array_equal(a[1], b[1])
        for i in range(len(Q)):
            assert g.decode_keys(a[0][i, : a[2][i]]) == h.decode_keys(b[0][i, : b[2][i]])
    assert h.export_bytes() == buf
    g.close()
    h.close()


def test_float_keys_match_rank_keys(H, O):
    rng = np.random.default_rng(17)
    n, d, M = 400, 10, 8
    keys = list(rng.normal(size=n) * 1e3)
    keys[0], keys[1], keys[2] = -0.0, 1e-300, -1e300
    X = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    lv = _levels(O, 0, M, 0.25, 20, 6, n)
    g = H.Graph(M=M, Ml=0.25, EfSearch=20, Distance=H.CosineDistance)
    g.BatchAdd([H.MakeNode(float(keys[i]), X[i]) for i in range(n)], levels=lv)
    Q = rng.uniform(-1, 1, (24, d)).astype(np.float32)
    _check_against_rank_oracle(H, O, g, [float(k) for k in keys], X, lv, Q, 0, M)
    assert g.Search(X[5], 1, mode=H.MODE_EXACT)[0].Key == float(keys[5])
    g.close()
