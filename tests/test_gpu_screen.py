"""GPU: the fp16 screening copy (option "screen"; DESIGN.md §6, "The fp16
screening copy") never changes a beam search or a batched build.  Every result (keys, f32 distance bits, counts) with the screen
on must equal the screen-off search and the oracle's beam search, on data built
to sit at the screen's edges: exact distance ties (integer-valued rows),
duplicates, rows and queries outside the screen's validity range (huge, tiny,
zero), and queries equal to stored rows."""
import numpy as np
import pytest

from tests.test_gpu_parity import _clustered, _metric_fn, _same_results

pytestmark = pytest.mark.gpu


def _adversarial(rng, n, d, metric):
    X = _clustered(rng, n, d)
    X[1] = X[2]                                   # duplicates
    X[3] = X[2]
    X[4] = np.nextafter(X[2], np.float32(np.inf))  # 1-ulp neighbour of a duplicate
    X[10] *= np.float32(1e20)                     # outside [2^-50, 2^50]: never screened
    X[11] *= np.float32(1e-20)
    X[12] *= np.float32(2.0 ** 49)                # inside the range, near its edges
    X[13] *= np.float32(2.0 ** -49)
    X[20:40] = rng.integers(-1, 2, size=(20, d)).astype(np.float32)  # many exact ties
    if metric == 0:
        X[14] = 0.0                               # zero row: NaN cosine
    Q = _clustered(rng, 96, d)
    Q[0] = X[2]
    Q[1] = X[25]
    Q[2] = 0.0
    Q[3] *= np.float32(1e30)                      # |q| > 2^40: query not screened
    Q[4] *= np.float32(1e-30)
    Q[5:9] = rng.integers(-1, 2, size=(4, d)).astype(np.float32)
    return X, Q


def _search(g, Q, ef, H):
    return g.search_arrays(Q, 10, mode=H.MODE_BEAM, ef=ef)


# dims cover every lane-contiguous row-load width (VPL 1, 2, 3, 4, 6)
@pytest.mark.parametrize("metric,d,n", [(0, 64, 20000), (1, 64, 20000), (0, 768, 6000), (1, 200, 8000),
                                        (1, 512, 4000), (0, 1024, 3000), (1, 1536, 2500)])
def test_screen_identical_to_f32(H, O, metric, d, n):
    rng = np.random.default_rng(100 + metric + d)
    X, Q = _adversarial(rng, n, d, metric)
    g = H.Graph(M=16, Ml=0.25, EfSearch=64, Distance=_metric_fn(H, metric), Rng=5, build_mode=H.BUILD_BATCH,
                ef_construction=100, heuristic=2, keep_pruned=1)
    g.add_arrays(np.arange(n), X)
    assert g.get_option("screen") == 1
    o = O.Graph(metric=metric, order=O.ORDER_DEV, M=16, M0=32, Ml=0.25, EfSearch=64)
    o.import_graph(**g.export())
    for ef in (10, 64, 200):
        g.set_option("screen", 0)
        g.reset_stats()
        off = _search(g, Q, ef, H)
        st = g.stats()
        assert st["search_screened"] == 0 and st["search_f32_evals"] == st["search_dist_evals"]
        _same_results(*off, *o.search(Q, 10, mode=O.MODE_BEAM, ef=ef))
        g.set_option("screen", 1)
        g.reset_stats()
        on = _search(g, Q, ef, H)
        st = g.stats()
        assert st["search_screened"] > 0, st
        assert st["search_f32_evals"] < st["search_dist_evals"]
        _same_results(*on, *off)
    g.close()


def test_screen_follows_adds_and_import(H, O):
    screen = 1
    rng = np.random.default_rng(7)
    n, d = 6000, 96
    X, Q = _adversarial(rng, n, d, 0)
    g = H.Graph(M=12, Ml=0.3, EfSearch=48, Distance=H.CosineDistance, Rng=3, build_mode=H.BUILD_BATCH,
                ef_construction=64, heuristic=2)
    g.set_option("screen", 0)
    g.add_arrays(np.arange(n // 2), X[: n // 2])
    g.set_option("screen", screen)                # enabling converts the rows already held
    g.add_arrays(np.arange(n // 2, n), X[n // 2:])  # later adds convert their own rows
    on = _search(g, Q, 48, H)
    g.set_option("screen", 0)
    _same_results(*on, *_search(g, Q, 48, H))
    # a graph rebuilt by Import screens the imported rows
    g2 = H.Graph(M=12, Ml=0.3, EfSearch=48, Distance=H.CosineDistance, Rng=3, build_mode=H.BUILD_BATCH,
                 screen=screen)
    g2.import_graph(**g.export())
    g2.reset_stats()
    _same_results(*on, *_search(g2, Q, 48, H))
    assert g2.stats()["search_screened"] > 0
    g.close()
    g2.close()


def test_screen_follows_metric_change(H, O):
    """Distance is a public field (graph.go:309): switching it rewrites the
    screening copy in the new metric's format."""
    rng = np.random.default_rng(8)
    n, d = 5000, 128
    X, Q = _adversarial(rng, n, d, 1)
    g = H.Graph(M=12, Ml=0.3, EfSearch=48, Distance=H.CosineDistance, Rng=3, build_mode=H.BUILD_BATCH,
                ef_construction=64, heuristic=2, screen=1)
    g.add_arrays(np.arange(n), X)
    for dist, metric in ((H.EuclideanDistance, 1), (H.CosineDistance, 0)):
        g.Distance = dist
        g.reset_stats()
        on = _search(g, Q, 48, H)
        assert g.stats()["search_screened"] > 0
        o = O.Graph(metric=metric, order=O.ORDER_DEV, M=12, M0=24, Ml=0.3, EfSearch=48)
        o.import_graph(**g.export())
        _same_results(*on, *o.search(Q, 10, mode=O.MODE_BEAM, ef=48))
        g.set_option("screen", 0)
        _same_results(*on, *_search(g, Q, 48, H))
        g.set_option("screen", 1)
    g.close()


@pytest.mark.parametrize("metric,alpha", [(0, 100), (1, 100), (0, 115), (1, 130)])
def test_screened_batch_build_identical(H, metric, alpha):
    """The batched insert's searches and its neighbour selection (the diversity
    rule with slack alpha, screened two-sided) screen too, and its greedy
    descents run in one launch per batch (fuse_descent): every combination
    builds the same graph as the plain per-layer, unscreened insert."""
    from tests.test_gpu_parity import _same_graph

    rng = np.random.default_rng(21 + metric)
    n, d = 12000, 96
    X, _ = _adversarial(rng, n, d, metric)
    ex, f32 = {}, {}
    for screen, fuse in ((0, 0), (1, 0), (0, 1), (1, 1)):
        g = H.Graph(M=12, Ml=0.3, EfSearch=48, Distance=_metric_fn(H, metric), Rng=3, build_mode=H.BUILD_BATCH,
                    ef_construction=80, heuristic=2, keep_pruned=1, screen=screen, fuse_descent=fuse,
                    prune_alpha_pct=alpha)
        g.add_arrays(np.arange(n // 3), X[: n // 3])   # two calls: later batches descend a multi-layer graph
        g.add_arrays(np.arange(n // 3, n), X[n // 3:])
        st = g.stats()
        assert st["dropped_proposals"] == 0
        f32[(screen, fuse)] = st["build_f32_rows"]
        ex[(screen, fuse)] = g.export()
        g.close()
    for key in ((1, 0), (0, 1), (1, 1)):
        _same_graph(ex[(0, 0)], ex[key])
    assert f32[(1, 0)] < 0.6 * f32[(0, 0)]  # the selection's rows were mostly decided on the copy
    # the 4-wave insert kernel (k_batch_search_mw: the screened searches' narrow launches by
    # default) on every launch, and on none: the same graph again
    for mw in (1 << 30, 0):
        g = H.Graph(M=12, Ml=0.3, EfSearch=48, Distance=_metric_fn(H, metric), Rng=3, build_mode=H.BUILD_BATCH,
                    ef_construction=80, heuristic=2, keep_pruned=1, screen=1, prune_alpha_pct=alpha,
                    build_mw_max=mw)
        g.add_arrays(np.arange(n // 3), X[: n // 3])
        g.add_arrays(np.arange(n // 3, n), X[n // 3:])
        _same_graph(ex[(0, 0)], g.export())
        g.close()
    # the insert searches' visited set at efConstruction 300 (> 128): the compact 16-bit
    # one (vis_compact, default) and the 32-bit one -- the same graph
    exv = []
    for c in (1, 0):
        g = H.Graph(M=12, Ml=0.3, EfSearch=48, Distance=_metric_fn(H, metric), Rng=3, build_mode=H.BUILD_BATCH,
                    ef_construction=300, heuristic=2, keep_pruned=1, screen=1, prune_alpha_pct=alpha, vis_compact=c)
        g.add_arrays(np.arange(n // 3), X[: n // 3])
        g.add_arrays(np.arange(n // 3, n), X[n // 3:])
        exv.append(g.export())
        g.close()
    _same_graph(exv[0], exv[1])
    # 1, 3 and 4 entries expanded per step of the insert's layer searches (build_expand; 4 is
    # what bench.py builds its indexes with): different graphs, but each the same with and
    # without the screen, and with the narrow launches on the 4-wave kernel (build_mw_max,
    # which covers every launch of this small build) or on the one-wave kernel
    for xw in (1, 3, 4):
        ex2 = []
        for screen, mw in ((0, 256), (1, 256), (1, 0), (1, 1 << 30)):
            g = H.Graph(M=12, Ml=0.3, EfSearch=48, Distance=_metric_fn(H, metric), Rng=3, build_mode=H.BUILD_BATCH,
                        ef_construction=80, heuristic=2, keep_pruned=1, screen=screen, prune_alpha_pct=alpha,
                        build_expand=xw, build_mw_max=mw)
            g.add_arrays(np.arange(n // 3), X[: n // 3])
            g.add_arrays(np.arange(n // 3, n), X[n // 3:])
            assert g.stats()["dropped_proposals"] == 0
            ex2.append(g.export())
            g.close()
        for e in ex2[1:]:
            _same_graph(ex2[0], e)
    # batches of 20 % of the index (bench.py's schedule for the bench index and
    # configs[2]): again the same graph with and without the screen
    ex3 = []
    for screen in (0, 1):
        g = H.Graph(M=12, Ml=0.3, EfSearch=48, Distance=_metric_fn(H, metric), Rng=3, build_mode=H.BUILD_BATCH,
                    ef_construction=80, heuristic=2, keep_pruned=1, screen=screen, prune_alpha_pct=alpha,
                    batch_ratio_pct=20)
        g.add_arrays(np.arange(n // 3), X[: n // 3])
        g.add_arrays(np.arange(n // 3, n), X[n // 3:])
        ex3.append(g.export())
        g.close()
    _same_graph(ex3[0], ex3[1])


@pytest.mark.parametrize("d", [1024, 1536])
def test_batch_build_wide_lists(H, O, d):
    """The batched insert with the widest candidate list (efConstruction 400:
    8 registers per lane) at the configurations that evaluate 4 rows per wave
    step (1024-d, 1536-d): the same graph with and without the fp16 screen, and
    the oracle's beam search on it == the engine's."""
    rng = np.random.default_rng(700 + d)
    n = 3000
    X, Q = _adversarial(rng, n, d, 0)
    graphs = []
    for scr in (1, 0):
        g = H.Graph(M=16, Ml=0.25, EfSearch=64, Distance=H.CosineDistance, Rng=5, build_mode=H.BUILD_BATCH,
                    ef_construction=400, heuristic=2, keep_pruned=1, m0=32, screen=scr)
        g.add_arrays(np.arange(n), X)
        graphs.append(g)
    ea, eb = graphs[0].export(), graphs[1].export()
    for name in ("deg", "adj", "entry"):
        assert np.array_equal(ea[name], eb[name]), name
    o = O.Graph(metric=O.COSINE, order=O.ORDER_DEV, M=16, M0=32, Ml=0.25, EfSearch=64)
    o.import_graph(**ea)
    _same_results(*_search(graphs[0], Q, 64, H), *o.search(Q, 10, mode=O.MODE_BEAM, ef=64))
    for g in graphs:
        g.close()
