"""CPU: the test-side restatement of encode.go (tests/go_format.py) against the
reference's own encoding tests, and Go-format round trips through the oracle
(TestGraph_ExportImport, encode_test.go:120-160, on the restatement)."""
import numpy as np
import pytest

from tests import go_format as F


def test_binary_varint():
    """encode_test.go:11-33 Test_binaryVarint: 1337 takes 2 bytes and the
    reader does not read past the varint."""
    b = F.put_varint(1337)
    assert len(b) == 2
    buf = b + bytes([0, 0, 0, 0])
    v, pos = F.read_varint(buf, 0)
    assert v == 1337 and buf[pos:] == bytes([0, 0, 0, 0])


def test_binary_write_string():
    """encode_test.go:35-50 Test_binaryWrite_string: 5 bytes + 1 length byte."""
    b = F.put_string("hello")
    assert len(b) == 6
    n, pos = F.read_varint(b, 0)
    assert b[pos:pos + n].decode() == "hello" and pos + n == len(b)


@pytest.mark.parametrize("x", [0, 1, -1, 63, -64, 64, 1 << 40, -(1 << 62), (1 << 63) - 1, -(1 << 63)])
def test_varint_zigzag_round_trip(x):
    v, pos = F.read_varint(F.put_varint(x), 0)
    assert v == x
    assert F.put_varint(-1) == b"\x01" and F.put_varint(1) == b"\x02"


def test_decode_errors():
    with pytest.raises(F.GoError, match=r"reading \*int at index 0: EOF"):
        F.decode(b"")
    good = F.encode(6, 0.5, 20, "euclidean", [[(1, np.ones(2), [])]])
    with pytest.raises(F.GoError, match='unknown distance function "manhattan"'):
        F.decode(F.encode(6, 0.5, 20, "manhattan", []))
    bad_version = F.put_varint(2) + good[1:]
    with pytest.raises(F.GoError, match="incompatible encoding version: 2"):
        F.decode(bad_version)
    assert F.decode(good)["layers"][0][0][0] == 1


def _oracle_graph(O, metric=1, n=128):
    g = O.Graph(metric=metric, order=O.ORDER_DEV, M=6, Ml=0.5, EfSearch=20)  # newTestGraph
    rng = np.random.default_rng(0)
    g.add(np.arange(n), rng.uniform(0, 1, (n, 1)).astype(np.float32))
    return g


def test_export_import_round_trip_oracle(O):
    """TestGraph_ExportImport on the restatement: Len, Topography,
    Connectivity and Search([0.5], 10) survive Export -> Import."""
    g1 = _oracle_graph(O)
    ex = g1.export()
    buf = F.encode_export(ex, 6, 0.5, 20, "euclidean")
    dec = F.decode(buf)
    assert (dec["M"], dec["Ml"], dec["EfSearch"], dec["dist"]) == (6, 0.5, 20, "euclidean")
    g2 = O.Graph(metric=O.EUCLIDEAN, order=O.ORDER_DEV, M=dec["M"], Ml=dec["Ml"], EfSearch=dec["EfSearch"])
    g2.import_graph(**F.to_csr(dec, ex["adj"].shape[2]))
    assert len(g2) == len(g1) and g2.topography() == g1.topography()
    q = np.array([[0.5]], np.float32)
    k1, d1, n1 = g1.search(q, 10)
    k2, d2, n2 = g2.search(q, 10)
    assert n1[0] == n2[0] and k1[0, : n1[0]].tolist() == k2[0, : n2[0]].tolist()
    # re-encoding the imported graph gives the same bytes (canonical order)
    assert F.encode_export(g2.export(), 6, 0.5, 20, "euclidean") == buf


def test_deleted_nodes_and_dangling_edges(O):
    """Deleted nodes are not written; edges pointing at them are (Go writes
    every map key) and resolve to nil on Import (dropped here)."""
    g = _oracle_graph(O, metric=0, n=200)
    g.delete(list(range(0, 200, 3)))
    ex = g.export()
    dec = F.decode(F.encode_export(ex, 6, 0.5, 20, "cosine"))
    live = {int(k) for k, d in zip(ex["keys"], ex["dead"]) if not d}
    assert {int(k) for k, _, _ in dec["layers"][0]} == live
    dangling = sum(1 for nodes in dec["layers"] for _, _, nbs in nodes for k in nbs if k not in live)
    csr = F.to_csr(dec, ex["adj"].shape[2])
    assert int(np.maximum(csr["deg"], 0).sum()) + dangling == sum(len(nbs) for nodes in dec["layers"]
                                                                    for _, _, nbs in nodes)
