"""GPU: the Python host mirror's Go-side behaviours that sit above the C ABI.

* Graph.Rng as a Go *rand.Rand (any object with Float64()): levels are drawn on
  the host by the reference rule (graph.go:388-417, layer-0 size growing per
  insert, across Add calls) and injected, so the graph depends on the caller's
  generator exactly as a Go graph does -- checked against the oracle built with
  the replayed levels.
* The opt-in dog-query hack of Search (graph.go:563-569, 595-619).
"""
import math

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


def _go_levels(draw, ml, n):
    """Independent restatement of graph.go:370-417 for n fresh inserts (layer 0
    of i nodes before insert i): maxLevel = Go math.Round(ln i / ln(1/ml)) + 1,
    halves away from zero (exact here: x.5 cases compare equal)."""
    out = []
    for i in range(n):
        if i == 0:
            mx = 1
        else:
            x = math.log(i) / math.log(1.0 / ml)
            f = math.floor(x)
            mx = int(f + 1 if x - f >= 0.5 else f) + 1
        lv = mx
        for level in range(mx):
            if draw() > ml:
                lv = level
                break
        out.append(lv)
    return out


class Scripted:
    """Float64() values from a list (a Go *rand.Rand stand-in with a known stream)"""

    def __init__(self, vals):
        self.vals, self.i = list(vals), 0

    def Float64(self):
        v = self.vals[self.i]
        self.i += 1
        return v


def test_host_rng_levels_build_the_oracle_graph(H, O):
    """Ml = 0.25 over 700 inserts crosses the layer-0 sizes where ln n / ln 4 is
    exactly x.5 (n = 2, 32, 512): there Go rounds the level cap up.  The graph
    built with a caller's Rng equals the oracle's built from levels of an
    independent restatement of the rule."""
    rng = np.random.default_rng(4)
    n, d, M, ml = 700, 20, 8, 0.25
    X = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    # a stream that stays below Ml for every draw at n = 2, 32, 512 (the cap
    # decides those levels) and is a generic LCG elsewhere
    special = {2, 32, 512}
    lcg = Lcg(99)
    vals = []
    for i in range(n):
        mx = 1 if i == 0 else int(math.floor(math.log(i) / math.log(4.0) + 0.5)) + 1
        for _ in range(mx):
            vals.append(0.1 if i in special else lcg.Float64())
            if vals[-1] > ml:
                break
    want = _go_levels(Scripted(vals).Float64, ml, n)
    assert [want[i] for i in sorted(special)] == [2, 4, 6]  # maxLevel(0.25, 2 / 32 / 512)
    g = H.Graph(M=M, Ml=ml, EfSearch=20, Distance=H.EuclideanDistance, Rng=Scripted(vals))
    g.BatchAdd([H.MakeNode(i, X[i]) for i in range(40)])
    for i in range(40, 60):
        g.Add(H.MakeNode(i, X[i]))
    g.add_arrays(np.arange(60, n), X[60:])
    o = O.Graph(metric=O.EUCLIDEAN, order=O.ORDER_DEV, M=M, Ml=ml, EfSearch=20)
    o.add(np.arange(n), X, np.array(want, np.int32))
    assert len(o.topography()) >= 6
    _same_graph(g.export(), o.export())
    assert g.Topography() == o.topography()
    # SplitMix64Rand(s) is the engine's own seed-s stream, and the engine's own
    # draws follow the same rule
    sm = H.SplitMix64Rand(42)
    st = [42]

    def splitmix():
        st[0] = (st[0] + 0x9E3779B97F4A7C15) & (2**64 - 1)
        z = st[0]
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & (2**64 - 1)
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & (2**64 - 1)
        return ((z ^ (z >> 31)) >> 11) / 9007199254740992.0

    want = _go_levels(splitmix, 0.25, 600)
    assert H.Graph(Rng=42).preview_levels(600).tolist() == want
    assert [H.random_level(sm, 0.25, i > 0, i) for i in range(600)] == want
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


@pytest.mark.parametrize("mode", ["batch", "flat"])
def test_batched_add_rejects_present_keys(H, mode):
    """The batched and flat builds have no reference semantics for a present key
    (graph.go:1015-1024 replaces it in BatchAdd's walk; compat mode does that):
    they reject the whole Add -- a key repeated inside the batch (in increasing,
    decreasing or shuffled key order) or one the index already holds -- and
    leave the index as it was."""
    bm = H.BUILD_BATCH if mode == "batch" else H.BUILD_FLAT
    rng = np.random.default_rng(3)
    X = rng.normal(size=(600, 16)).astype(np.float32)
    g = H.Graph(M=8, Ml=0.25, EfSearch=20, Distance=H.EuclideanDistance, build_mode=bm)
    g.add_arrays(np.arange(0, 400, 2), X[:200])  # increasing keys: the map-free duplicate check
    assert len(g) == 200
    for keys in (np.array([1001, 1003, 1003, 1005]), np.array([1009, 1007, 1007, 1005]),
                 rng.permutation(np.array([1011, 1013, 1015, 1013])), np.array([2001, 2003, 4, 2005])):
        with pytest.raises(H.HnswError, match="duplicate key"):
            g.add_arrays(keys, X[200:200 + len(keys)])
        assert len(g) == 200
    g.add_arrays(np.array([3001, 3000, 3002]), X[300:303])  # not increasing, no repeat: accepted
    assert len(g) == 203
    gk, _, gn = g.search_arrays(X[300:303], 1, mode=H.MODE_EXACT)
    assert gk[:, 0].tolist() == [3001, 3000, 3002]
    g.close()
