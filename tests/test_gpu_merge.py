"""GPU: the batched list update of the query search's 256- and 512-entry lists
(device_search.hpp bl_merge, beam_layer MERGE): each layer-0 step's candidates
are merged into the list at once instead of one bl_insert each.  The list after
a step is the best ef of its entries and the step's candidates whatever the
order, so the results must equal the oracle's one-at-a-time restatement bit for
bit -- on the fast path (distinct distances), on the fallback taken when a
candidate's distance equals a listed one (duplicate rows: every vector stored
three times under different keys), for XW 1 / 2 / 4, both metrics, and with
the merge scratch placed after the compact set, after the 32-bit set, and after
a compact set given more LDS than the default.
"""
import numpy as np
import pytest

from tests.test_gpu_parity import _clustered, _metric_fn, _same_results

pytestmark = pytest.mark.gpu


def _graph(H, O, metric, X, seed):
    g = H.Graph(M=16, Ml=0.25, EfSearch=64, Distance=_metric_fn(H, metric), Rng=seed, build_mode=H.BUILD_BATCH,
                ef_construction=100, heuristic=2, m0=32)
    g.add_arrays(np.arange(len(X)) * 5 + 2, X)
    o = O.Graph(metric=metric, order=O.ORDER_DEV, M=16, M0=32, Ml=0.25, EfSearch=64)
    o.import_graph(**g.export())
    return g, o


@pytest.fixture(scope="module")
def dup_built(H, O):
    """rows stored three times each (equal distances in every list)"""
    out = {}
    for metric in (0, 1):
        rng = np.random.default_rng(71 + metric)
        base = _clustered(rng, 3000, 48, intrinsic=16)
        X = np.repeat(base, 3, axis=0)
        Q = _clustered(rng, 96, 48, intrinsic=16)
        out[metric] = (*_graph(H, O, metric, X, 9), Q)
    yield out
    for g, _, _ in out.values():
        g.close()


def _check(H, O, g, o, Q, xw, ef, **opts):
    o.set_search_expand(xw)
    rk, rd, rn = o.search(Q, 10, mode=O.MODE_BEAM, ef=ef)
    o.set_search_expand(1)
    old = {k: g.get_option(k) for k in ("search_expand", *opts)}
    try:
        g.set_option("search_expand", xw)
        for k, v in opts.items():
            g.set_option(k, v)
        gk, gd, gn = g.search_arrays(Q, 10, mode=H.MODE_BEAM, ef=ef)
        _same_results(gk, gd, gn, rk, rd, rn)
    finally:
        for k, v in old.items():
            g.set_option(k, v)


@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("xw", [1, 2, 4])
@pytest.mark.parametrize("ef", [129, 256, 300, 512])
def test_merge_duplicate_rows(H, O, dup_built, metric, xw, ef):
    g, o, Q = dup_built[metric]
    _check(H, O, g, o, Q, xw, ef)


@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("xw", [1, 4])
def test_merge_scratch_placements(H, O, metric, xw):
    """the scratch after the compact set (default), after the 32-bit set
    (vis_compact 0: the launch adds the scratch's LDS), and after a compact set
    whose LDS was raised to less than the set plus the scratch (vis_entries
    4,200 words)"""
    rng = np.random.default_rng(13 + metric)
    X = _clustered(rng, 12000, 64, intrinsic=20)
    Q = _clustered(rng, 64, 64, intrinsic=20)
    g, o = _graph(H, O, metric, X, 4)
    try:
        for ef in (200, 512):
            _check(H, O, g, o, Q, xw, ef)
            _check(H, O, g, o, Q, xw, ef, vis_compact=0)
            _check(H, O, g, o, Q, xw, ef, vis_entries=4200)
    finally:
        g.close()
