"""GPU: the Python host mirror's Go-side behaviours that sit above the C ABI.

* Graph.Rng as a Go *rand.Rand (any object with Float64()): levels are drawn on
  the host by the reference rule (graph.go:388-417, layer-0 size growing per
  insert, across Add calls) and injected, so the graph depends on the caller's
  generator exactly as a Go graph does -- checked against the oracle built with
  the replayed levels.
* The opt-in dog-query hack of Search (graph.go:563-569, 595-619).
"""
import numpy as np
import pytest

from tests.test_gpu_parity import _same_graph

pytestmark = pytest.mark.gpu


class Lcg:
    """a caller-supplied generator, not the engine's stream"""

    def __init__(self, s):
        self.s = s

    def Float64(self):
        self.s = (self.s * 6364136223846793005 + 1442695040888963407) & (2**64 - 1)
        return (self.s >> 11) / 9007199254740992.0


def test_host_rng_levels_build_the_oracle_graph(H, O):
    from hnsw_amd.graph import random_level

    rng = np.random.default_rng(4)
    n, d, M, ml = 700, 20, 8, 0.3
    X = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    g = H.Graph(M=M, Ml=ml, EfSearch=20, Distance=H.EuclideanDistance, Rng=Lcg(99))
    g.BatchAdd([H.MakeNode(i, X[i]) for i in range(40)])
    for i in range(40, 60):
        g.Add(H.MakeNode(i, X[i]))
    g.add_arrays(np.arange(60, n), X[60:])
    r = Lcg(99)
    lv = np.array([random_level(r, ml, i > 0, i) for i in range(n)], np.int32)
    o = O.Graph(metric=O.EUCLIDEAN, order=O.ORDER_DEV, M=M, Ml=ml, EfSearch=20)
    o.add(np.arange(n), X, lv)
    assert len(o.topography()) >= 3
    _same_graph(g.export(), o.export())
    # SplitMix64Rand(s) is the engine's own seed-s stream
    from hnsw_amd.graph import SplitMix64Rand

    sm = SplitMix64Rand(42)
    want = H.Graph(Rng=42).preview_levels(300)
    assert [random_level(sm, 0.25, i > 0, i) for i in range(300)] == want.tolist()
    g.close()


def test_dog_query_hack_opt_in(H):
    # hand graph (one layer): canine (key 3) unreachable from the entry
    keys = np.array([1, 2, 3, 4, 5], np.int64)  # dog, puppy, canine, cat, kitten (negative_test.go:17-23)
    vals = np.array([[1.0, 0.2, 0.1], [0.9, 0.3, 0.2], [0.8, 0.3, 0.3], [0.1, 1.0, 0.2], [0.2, 0.9, 0.3]], np.float32)
    deg = np.array([[2, 2, 0, 2, 2]], np.int32)
    adj = -np.ones((1, 5, 5), np.int32)
    adj[0, 0, :2] = [1, 3]
    adj[0, 1, :2] = [0, 4]
    adj[0, 3, :2] = [0, 4]
    adj[0, 4, :2] = [1, 3]
    g = H.Graph(M=4, Ml=0.5, EfSearch=20, Distance=H.CosineDistance)
    g.import_graph(keys, vals, deg, adj, np.array([0], np.int32))
    dog = [1.0, 0.2, 0.1]
    plain = [n.Key for n in g.Search(dog, 3)]
    assert len(plain) == 3 and 3 not in plain
    g.TestHacks = H.DOG_QUERY_HACK
    hacked = g.Search(dog, 3)
    assert [n.Key for n in hacked] == plain[:2] + [3]
    assert hacked[2].Value.tolist() == vals[2].tolist()
    assert 3 not in [n.Key for n in g.Search([1.0, 0.2, 0.1000001], 3)]  # not the dog query
    assert 3 not in [n.Key for n in g.BatchSearch([dog], 3)[0]]         # BatchSearch has no hack (graph.go:1047)
    g.close()
