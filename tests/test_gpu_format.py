"""GPU: the engine's Go-format codec (mhnsw_export_go / mhnsw_import_go /
mhnsw_save / mhnsw_load, encode.go:128-327) against the test-side
restatement tests/go_format.py, and the reference's encode tests."""
import io
import os

import numpy as np
import pytest

from tests import go_format as F
from tests.test_gpu_parity import _levels, _same_graph, _same_results

pytestmark = pytest.mark.gpu


def _compat_graph(H, O, n=500, d=16, metric=0, M=8, deletes=0, seed=1):
    rng = np.random.default_rng(seed)
    X = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    lv = _levels(O, metric, M, 0.25, 20, 7, n)
    g = H.Graph(M=M, Ml=0.25, EfSearch=20, Distance=H.CosineDistance if metric == 0 else H.EuclideanDistance)
    g.add_arrays(np.arange(n) * 7 - 100, X, levels=lv)
    if deletes:
        g.BatchDelete([int(k) for k in rng.choice(np.arange(n) * 7 - 100, deletes, replace=False)])
    return g, rng


@pytest.mark.parametrize("deletes", [0, 60])
@pytest.mark.parametrize("kind", [0, 1, 2])
def test_export_bytes_match_restatement(H, O, deletes, kind):
    g, _ = _compat_graph(H, O, deletes=deletes)
    ex = g.export()
    want = F.encode_export(ex, g.M, g.Ml, g.EfSearch, "cosine", kind)
    assert g.export_bytes(kind) == want


@pytest.mark.parametrize("metric", [0, 1])
def test_import_matches_oracle(H, O, metric):
    """A Go-format file (with dangling edges to deleted nodes) imported by the
    engine == the same file decoded by the restatement and imported by the
    oracle: identical graphs, identical compat/beam/exact results."""
    g, rng = _compat_graph(H, O, n=700, d=24, metric=metric, deletes=90, seed=3)
    buf = g.export_bytes()
    h = H.Graph()  # default parameters: the file's M/Ml/EfSearch/Distance win
    h.import_bytes(buf)
    assert (h.M, h.Ml, h.EfSearch) == (g.M, g.Ml, g.EfSearch)
    assert h.Distance is g.Distance
    dec = F.decode(buf)
    o = O.Graph(metric=metric, order=O.ORDER_DEV, M=dec["M"], Ml=dec["Ml"], EfSearch=dec["EfSearch"])
    ex = h.export()
    o.import_graph(**F.to_csr(dec, ex["adj"].shape[2]))
    _same_graph(ex, o.export())
    assert h.Len() == g.Len() and h.Topography() == g.Topography()
    Q = rng.uniform(-1, 1, (40, 24)).astype(np.float32)
    for mode in (H.MODE_COMPAT, H.MODE_BEAM, H.MODE_EXACT):
        gk, gd, gn = h.search_arrays(Q, 10, mode=mode, ef=32)
        rk, rd, rn = o.search(Q, 10, mode=mode, ef=32)
        _same_results(gk, gd, gn, rk, rd, rn)
    # re-export: same nodes, dangling neighbour keys dropped, else unchanged
    want = [{k: [x for x in v if x in layer] for k, v in layer.items()} for layer in F.structure(dec)]
    assert F.structure(F.decode(h.export_bytes())) == want


def test_graph_export_import(H):
    """encode_test.go:120-160 TestGraph_ExportImport (newTestGraph: M=6,
    Ml=0.5, EfSearch=20, Euclidean; 128 1-D nodes)."""
    rng = np.random.default_rng(0)
    g1 = H.Graph(M=6, Ml=0.5, EfSearch=20, Distance=H.EuclideanDistance, Rng=0)
    for i in range(128):
        g1.Add(H.MakeNode(i, rng.uniform(0, 1, 1).astype(np.float32)))
    buf = io.BytesIO()
    g1.Export(buf)
    buf.seek(0)
    g2 = H.Graph()
    g2.Import(buf)
    assert g1.Len() == g2.Len() and g1.Topography() == g2.Topography()
    assert g1.Connectivity() == g2.Connectivity()
    assert g1.Distance([0.5], [1]) == g2.Distance([0.5], [1])
    assert (g1.M, g1.Ml, g1.EfSearch) == (g2.M, g2.Ml, g2.EfSearch)
    n1 = g1.Search([0.5], 10)
    n2 = g2.Search([0.5], 10)
    assert [n.Key for n in n1] == [n.Key for n in n2]
    assert all(np.array_equal(a.Value, b.Value) for a, b in zip(n1, n2))


def test_saved_graph(H, tmp_path):
    """encode_test.go:162-183 TestSavedGraph."""
    path = str(tmp_path / "graph")
    g1 = H.LoadSavedGraph(path)
    assert g1.Len() == 0
    rng = np.random.default_rng(1)
    for i in range(128):
        g1.Add(H.MakeNode(i, rng.uniform(0, 1, 1).astype(np.float32)))
    g1.Save()
    g2 = H.LoadSavedGraph(path)
    assert g2.Len() == 128 and g1.Topography() == g2.Topography() and g1.Connectivity() == g2.Connectivity()
    assert (g1.M, g1.Ml, g1.EfSearch) == (g2.M, g2.Ml, g2.EfSearch)
    assert not os.path.exists(path + ".tmp")


def test_import_errors(H):
    g = H.Graph()
    with pytest.raises(H.HnswError, match=r"reading \*int at index 0: EOF"):
        g.import_bytes(b"")
    with pytest.raises(H.HnswError, match='unknown distance function "manhattan"'):
        g.import_bytes(F.encode(6, 0.5, 20, "manhattan", []))
    good = F.encode(6, 0.5, 20, "euclidean", [[(1, np.ones(2), [2]), (2, np.zeros(2), [1])]])
    with pytest.raises(H.HnswError, match="incompatible encoding version: 2"):
        g.import_bytes(F.put_varint(2) + good[1:])
    with pytest.raises(H.HnswError, match="decoding neighbor 0 for node 1: EOF"):
        g.import_bytes(good[:-1])
    g.import_bytes(good)
    assert g.Len() == 2 and g.Dims() == 2


def test_batch_graph_round_trip(H):
    """A batched-build graph survives Export/Import with identical beam and
    exact results (row order changes to ascending keys; results do not)."""
    rng = np.random.default_rng(5)
    X = rng.normal(size=(20000, 64)).astype(np.float32)
    g = H.Graph(M=16, EfSearch=64, Rng=2, build_mode=H.BUILD_BATCH, m0=32, ef_construction=100, heuristic=2)
    g.add_arrays(np.arange(20000), X)
    h = H.Graph(build_mode=H.BUILD_BATCH, m0=32)
    h.import_bytes(g.export_bytes(H.KEY_INT64), H.KEY_INT64)
    Q = rng.normal(size=(300, 64)).astype(np.float32)
    for mode, ef in ((H.MODE_BEAM, 64), (H.MODE_EXACT, 0)):
        a = g.search_arrays(Q, 10, mode=mode, ef=ef)
        b = h.search_arrays(Q, 10, mode=mode, ef=ef)
        _same_results(*a, *b)
