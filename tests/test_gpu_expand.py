"""GPU: the beam search with several entries expanded per layer-0 step
(option "search_expand" 2 / 4; device_search.hpp beam_layer XW, beam.hpp).

A wider step is a different search from the standard one (the second entry is
expanded before the first one's neighbours can displace it), so its results are
compared with the oracle's restatement of the same search
(oracle.c beam_layer_search with og_set_search_expand): bit-identical keys,
counts and distances, with the fp16 screen on and off, with the compact and the
32-bit visited set, with sets small enough to forget on every query, for single
queries and for batches, and after deletions.
"""
import numpy as np
import pytest

from tests.test_gpu_parity import _clustered, _metric_fn, _same_results

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def built(H, O):
    """one batched graph per metric, mirrored into the oracle"""
    out = {}
    for metric in (0, 1):
        rng = np.random.default_rng(41 + metric)
        n, d = 20000, 96
        X = _clustered(rng, n, d, intrinsic=24)
        Q = _clustered(rng, 128, d, intrinsic=24)
        g = H.Graph(M=16, Ml=0.25, EfSearch=64, Distance=_metric_fn(H, metric), Rng=5, build_mode=H.BUILD_BATCH,
                    ef_construction=100, heuristic=2, m0=32)
        g.add_arrays(np.arange(n) * 3 + 1, X)
        o = O.Graph(metric=metric, order=O.ORDER_DEV, M=16, M0=32, Ml=0.25, EfSearch=64)
        o.import_graph(**g.export())
        out[metric] = (g, o, Q)
    yield out
    for g, _, _ in out.values():
        g.close()


def _with(g, **opts):
    old = {k: g.get_option(k) for k in opts}
    for k, v in opts.items():
        g.set_option(k, v)
    return old


@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("xw", [2, 4])
@pytest.mark.parametrize("ef", [10, 64, 200, 512])
def test_search_expand_matches_oracle(H, O, built, metric, xw, ef):
    g, o, Q = built[metric]
    o.set_search_expand(xw)
    rk, rd, rn = o.search(Q, 10, mode=O.MODE_BEAM, ef=ef)
    o.set_search_expand(1)
    old = _with(g, search_expand=xw)
    try:
        for screen in (1, 0):
            for compact in (1, 0):
                _with(g, screen=screen, vis_compact=compact)
                gk, gd, gn = g.search_arrays(Q, 10, mode=H.MODE_BEAM, ef=ef)
                _same_results(gk, gd, gn, rk, rd, rn)
    finally:
        _with(g, screen=1, vis_compact=1, **old)


@pytest.mark.parametrize("metric", [0, 1])
def test_search_expand_is_a_different_search(H, O, built, metric):
    """XW 2 / 4 expand more entries than XW 1 (the step's second entry is taken
    before the first one's neighbours arrive) and the oracle counts the same
    expansions; at ef 200 on this graph the lists of the three searches are not
    all identical, and their recall is the same within 2 %."""
    g, o, Q = built[metric]
    ek, _, en = g.search_arrays(Q, 10, mode=H.MODE_EXACT)
    res, xs = {}, {}
    for xw in (1, 2, 4):
        _with(g, search_expand=xw)
        g.reset_stats()
        res[xw] = g.search_arrays(Q, 10, mode=H.MODE_BEAM, ef=200)
        xs[xw] = g.stats()["search_expansions"]
        o.set_search_expand(xw)
        x0 = o.stats()[1]
        o.search(Q, 10, mode=O.MODE_BEAM, ef=200)
        assert o.stats()[1] - x0 == xs[xw], (xw, o.stats()[1] - x0, xs)
    o.set_search_expand(1)
    _with(g, search_expand=1)
    assert xs[1] <= xs[2] <= xs[4], xs
    rec = {xw: np.mean([len(set(r[0][b, : r[2][b]]) & set(ek[b, : en[b]])) / 10 for b in range(len(Q))])
           for xw, r in res.items()}
    assert max(rec.values()) - min(rec.values()) <= 0.02, rec


@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("xw", [2, 4])
def test_search_expand_forgetting(H, O, built, metric, xw):
    """visited sets small enough to reset on every query: still the oracle's
    results (which never forget)"""
    g, o, Q = built[metric]
    o.set_search_expand(xw)
    rk, rd, rn = o.search(Q, 10, mode=O.MODE_BEAM, ef=128)
    o.set_search_expand(1)
    old = _with(g, search_expand=xw)
    try:
        for vis_log2 in (6, 8):
            _with(g, vis_log2=vis_log2)
            g.reset_stats()
            gk, gd, gn = g.search_arrays(Q, 10, mode=H.MODE_BEAM, ef=128)
            assert g.stats()["visited_resets"] >= len(Q)
            _same_results(gk, gd, gn, rk, rd, rn)
    finally:
        _with(g, vis_log2=12, **old)


@pytest.mark.parametrize("xw", [2, 4])
def test_search_expand_small_batches(H, O, built, xw):
    """batches below beam_mw_max_b run the one-wave kernel at XW > 1 (the
    4-wave small-batch kernel is the standard search): B = 1 and B = 7 equal
    the oracle and the same queries inside the full batch"""
    g, o, Q = built[0]
    o.set_search_expand(xw)
    rk, rd, rn = o.search(Q, 10, mode=O.MODE_BEAM, ef=64)
    o.set_search_expand(1)
    old = _with(g, search_expand=xw)
    try:
        for lo, hi in ((0, 1), (5, 12)):
            gk, gd, gn = g.search_arrays(Q[lo:hi], 10, mode=H.MODE_BEAM, ef=64)
            _same_results(gk, gd, gn, rk[lo:hi], rd[lo:hi], rn[lo:hi])
    finally:
        _with(g, **old)


def test_search_expand_after_deletes(H, O):
    """deleted rows route the search but are never returned, at XW 4 as at XW 1"""
    rng = np.random.default_rng(5)
    n, d = 6000, 40
    X = _clustered(rng, n, d)
    Q = _clustered(rng, 64, d)
    g = H.Graph(M=12, Ml=0.25, EfSearch=64, Distance=H.CosineDistance, Rng=3, build_mode=H.BUILD_BATCH,
                ef_construction=80, heuristic=2, m0=24)
    g.add_arrays(np.arange(n), X)
    g.BatchDelete(list(range(0, n, 7)))
    o = O.Graph(metric=O.COSINE, order=O.ORDER_DEV, M=12, M0=24, Ml=0.25, EfSearch=64)
    o.import_graph(**g.export())
    g.set_option("search_expand", 4)
    o.set_search_expand(4)
    for ef in (32, 150):
        gk, gd, gn = g.search_arrays(Q, 10, mode=H.MODE_BEAM, ef=ef)
        rk, rd, rn = o.search(Q, 10, mode=O.MODE_BEAM, ef=ef)
        _same_results(gk, gd, gn, rk, rd, rn)
        assert not (set(gk[gk >= 0].tolist()) & set(range(0, n, 7)))
    g.close()


def test_search_expand_option_values(H):
    g = H.Graph(M=8, Ml=0.25, EfSearch=20, Distance=H.CosineDistance)
    assert g.get_option("search_expand") == 1
    for bad in (0, 3, 5):
        with pytest.raises(H.HnswError, match="search_expand must be 1, 2 or 4"):
            g.set_option("search_expand", bad)
    g.set_option("search_expand", 2)
    assert g.get_option("search_expand") == 2
    g.close()
