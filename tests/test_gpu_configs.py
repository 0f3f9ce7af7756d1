"""GPU: BASELINE configs[0] at its stated size, against the oracle.

configs[0] = "10k x 128-d random float32, CosineDistance, M=16 efSearch=20,
pure-Go CPU Search (graph_benchmark_test.go path)"; data as SURVEY §8(d) C1:
X ~ U[-1,1) (graph_benchmark_test.go:12-18), seed 42, then 1000 queries from
the same stream; Ml = 0.25, k = 10.  The engine runs the reference's own
semantics end to end -- compat build (graph.go:437-531, levels from the
engine's seed-42 stream, injected into the oracle) and compat Search
(graph.go:534-625) -- and must reproduce the restatement exactly: the same
graph, the same keys in the same (heap) order, bit-identical distances.
"""
import numpy as np
import pytest

from oracle.parity import compare_lists, same_graph
from tests.test_gpu_parity import _same_graph, _same_results

pytestmark = pytest.mark.gpu


def test_config0_fullsize_compat_build_and_search(H, O):
    rng = np.random.default_rng(42)
    n, d, nq, k = 10_000, 128, 1000, 10
    X = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    Q = rng.uniform(-1, 1, (nq, d)).astype(np.float32)
    keys = np.arange(n, dtype=np.int64)
    g = H.Graph(M=16, Ml=0.25, EfSearch=20, Distance=H.CosineDistance, Rng=42)
    lv = g.preview_levels(n)
    g.add_arrays(keys, X)
    o = O.Graph(metric=O.COSINE, order=O.ORDER_DEV, M=16, Ml=0.25, EfSearch=20)
    o.add(keys, X, lv)
    assert g.Topography() == o.topography()
    _same_graph(g.export(), o.export())
    # the reference's Search(): identical keys in heap order, bit-identical distances
    gk, gd, gn = g.search_arrays(Q, k, mode=H.MODE_COMPAT)
    rk, rd, rn = o.search(Q, k, mode=O.MODE_COMPAT)
    _same_results(gk, gd, gn, rk, rd, rn)
    # beam and exact on the same graph
    for mode in (H.MODE_BEAM, H.MODE_EXACT):
        bk, bd, bn = g.search_arrays(Q, k, mode=mode, ef=20)
        ok, od, on = o.search(Q, k, mode=mode, ef=20)
        _same_results(bk, bd, bn, ok, od, on)
    # recall of the reference algorithm on this data (SURVEY A.3 simulated 0.022)
    ek, _, en = o.search(Q, k, mode=O.MODE_EXACT)
    rec = np.mean([len(set(gk[b, : gn[b]]) & set(ek[b, : en[b]])) / k for b in range(nq)])
    assert 0.005 < rec < 0.08, rec
    # ORDER_REF: the reference's arithmetic, the reference's Add and Search
    r = O.Graph(metric=O.COSINE, order=O.ORDER_REF, M=16, Ml=0.25, EfSearch=20)
    r.add(keys, X, lv)
    assert same_graph(g.export(), r.export())
    pr = compare_lists((gk, gd, gn), r.search(Q, k, mode=O.MODE_COMPAT), k, truth=(ek, en))
    print("configs[0] GPU compat vs ORDER_REF:", pr)
    assert pr["recall_delta"] <= 0.002 and pr["max_abs_dist_diff"] <= 1e-5, pr
    assert pr["identical_lists"] >= 0.99, pr
    g.close()
