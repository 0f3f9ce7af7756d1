"""GPU: the small-batch beam kernel (k_search_beam_mw, beam.hpp: one workgroup
of 4 waves per query, the single-query latency path of ParallelSearch,
graph.go:631-790) returns exactly what the one-wave kernel and the oracle's
beam search return -- keys, f32 distance bits and counts -- on the screening
copy's edge cases (tests/test_gpu_screen.py _adversarial), with the screen on
and off, at B = 1 and B = 96, ef up to 128 (the kernel's list widths R = 1, 2)."""
import numpy as np
import pytest

from tests.test_gpu_parity import _metric_fn, _same_results
from tests.test_gpu_screen import _adversarial

pytestmark = pytest.mark.gpu


def _rows(res, i):
    return tuple(x[i:i + 1] for x in res)


# 64 / 128 / 768 / 1536-d: the 16-, 32-, 64-lane row maps and the 3- and 6-vector rows
@pytest.mark.parametrize("metric,d,n", [(0, 768, 6000), (1, 128, 12000), (0, 1536, 3000), (1, 64, 20000)])
def test_multiwave_beam_identical(H, O, metric, d, n):
    rng = np.random.default_rng(700 + metric + d)
    X, Q = _adversarial(rng, n, d, metric)
    g = H.Graph(M=16, Ml=0.25, EfSearch=64, Distance=_metric_fn(H, metric), Rng=5, build_mode=H.BUILD_BATCH,
                ef_construction=100, heuristic=2, keep_pruned=1)
    g.add_arrays(np.arange(n), X)
    assert g.get_option("beam_mw_max_b") == 512
    o = O.Graph(metric=metric, order=O.ORDER_DEV, M=16, M0=32, Ml=0.25, EfSearch=64)
    o.import_graph(**g.export())
    for screen in (1, 0):
        g.set_option("screen", screen)
        for ef in (10, 64, 128):
            g.set_option("beam_mw_max_b", 0)
            one_wave = g.search_arrays(Q, 10, mode=H.MODE_BEAM, ef=ef)
            g.set_option("beam_mw_max_b", 512)
            multi = g.search_arrays(Q, 10, mode=H.MODE_BEAM, ef=ef)
            _same_results(*multi, *one_wave)
            _same_results(*multi, *o.search(Q, 10, mode=O.MODE_BEAM, ef=ef))
            for i in (0, 3, 5, 40):
                _same_results(*g.search_arrays(Q[i:i + 1], 10, mode=H.MODE_BEAM, ef=ef), *_rows(multi, i))


def test_multiwave_beam_after_deletes(H, O):
    """Deleted rows route the search but are never returned: the same in both kernels."""
    rng = np.random.default_rng(71)
    n, d = 8000, 256
    X = rng.standard_normal((n, d)).astype(np.float32)
    Q = rng.standard_normal((64, d)).astype(np.float32)
    g = H.Graph(M=16, Ml=0.25, EfSearch=64, Distance=H.CosineDistance, Rng=5, build_mode=H.BUILD_BATCH,
                ef_construction=100, heuristic=2, keep_pruned=1)
    g.add_arrays(np.arange(n), X)
    g.BatchDelete([int(k) for k in rng.choice(n, 800, replace=False)])
    g.set_option("beam_mw_max_b", 0)
    one_wave = g.search_arrays(Q, 10, mode=H.MODE_BEAM, ef=64)
    g.set_option("beam_mw_max_b", 512)
    _same_results(*g.search_arrays(Q, 10, mode=H.MODE_BEAM, ef=64), *one_wave)
