"""GPU: the visited set's two behaviours.

Beam mode may *forget*: once the LDS set is 3/4 full it is cleared
(device_search.hpp beam_layer), and a node seen before can be evaluated again.
DESIGN.md §6 argues the results cannot change -- a re-evaluated node either
sits in the sorted list already (its (dist, id) is rejected as a duplicate) or
was rejected before against a worst entry that has only decreased since.  The
oracle's beam search (oracle.c beam_layer_search) never forgets, so running the
GPU with tiny sets (2^6..2^8 entries, resets on every query) against it checks
that argument directly, screen on and off.

Compat mode needs the exact set (graph.go:141-144 keeps a map): an overflow is
an error.  Asynchronous *_device searches surface it through
mhnsw_device_status; synchronous calls (host search, negatives) return it.
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
        rng = np.random.default_rng(31 + metric)
        n, d = 12000, 48
        X = _clustered(rng, n, d)
        Q = _clustered(rng, 96, d)
        g = H.Graph(M=12, Ml=0.25, EfSearch=64, Distance=_metric_fn(H, metric), Rng=5, build_mode=H.BUILD_BATCH,
                    ef_construction=80, heuristic=2, m0=24)
        g.add_arrays(np.arange(n) * 3 + 1, X)
        o = O.Graph(metric=metric, order=O.ORDER_DEV, M=12, M0=24, Ml=0.25, EfSearch=64)
        o.import_graph(**g.export())
        out[metric] = (g, o, Q)
    yield out
    for g, _, _ in out.values():
        g.close()


@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("vis_log2", [6, 7, 8])
@pytest.mark.parametrize("ef", [64, 200])
def test_beam_forgetting_matches_oracle(H, O, built, metric, vis_log2, ef):
    g, o, Q = built[metric]
    rk, rd, rn = o.search(Q, 10, mode=O.MODE_BEAM, ef=ef)
    for screen in (1, 0):
        g.set_option("screen", screen)
        g.set_option("vis_log2", vis_log2)
        g.reset_stats()
        gk, gd, gn = g.search_arrays(Q, 10, mode=H.MODE_BEAM, ef=ef)
        st = g.stats()
        g.set_option("vis_log2", 12)
        # every query forgets at least once with sets this small
        assert st["visited_resets"] >= len(Q), st
        _same_results(gk, gd, gn, rk, rd, rn)
    g.set_option("screen", 1)


def test_beam_forgetting_costs_only_evaluations(H, built):
    """same results, more distance evaluations with the smaller set"""
    g, _, Q = built[0]
    evals = {}
    res = {}
    for v in (12, 7):
        g.set_option("vis_log2", v)
        g.reset_stats()
        res[v] = g.search_arrays(Q, 10, mode=H.MODE_BEAM, ef=200)
        st = g.stats()
        evals[v] = st["search_dist_evals"]
        if v == 12:
            assert st["visited_resets"] == 0, st  # the full-size set never fills here
    g.set_option("vis_log2", 12)
    for a, b in zip(res[12], res[7]):
        assert np.array_equal(a, b)
    assert evals[7] > 1.1 * evals[12], evals


def _compat_overflow_graph(H, O):
    rng = np.random.default_rng(77)
    n, d = 4000, 8
    X = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    lv = O.Graph(metric=O.COSINE, M=16, Ml=0.25, EfSearch=20, seed=3).preview_levels(n)
    g = H.Graph(M=16, Ml=0.25, EfSearch=20, Distance=H.CosineDistance)
    g.add_arrays(np.arange(n), X, levels=lv)
    Q = rng.uniform(-1, 1, (32, d)).astype(np.float32)
    return g, Q


def test_compat_overflow_reported_everywhere(H, O):
    torch = pytest.importorskip("torch")
    g, Q = _compat_overflow_graph(H, O)
    k, ef = 200, 400
    # a set of 2^13 holds it (at most 4000 nodes)
    g.set_option("vis_log2", 13)
    gk, gd, gn = g.search_arrays(Q, k, mode=H.MODE_COMPAT, ef=ef)
    assert gn.min() > 0
    g.set_option("vis_log2", 6)
    # synchronous host-pointer search
    with pytest.raises(H.HnswError, match="visited set overflow"):
        g.search_arrays(Q, k, mode=H.MODE_COMPAT, ef=ef)
    # negatives: the candidate search (kx = 3k) reports too
    negs = [Q[(i + 1) % len(Q)][None] for i in range(len(Q))]
    with pytest.raises(H.HnswError, match="visited set overflow"):
        g.search_negatives_arrays(Q, negs, 60, 0.5, mode=H.MODE_COMPAT, ef=ef)
    # asynchronous device search: enqueued fine, the status call reports it once
    dev = torch.device("cuda:0")
    dq = torch.from_numpy(Q).to(dev)
    ok = torch.empty((len(Q), k), dtype=torch.int64, device=dev)
    od = torch.empty((len(Q), k), dtype=torch.float32, device=dev)
    on = torch.empty((len(Q),), dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    g.search_device(dq.data_ptr(), len(Q), Q.shape[1], k, ok.data_ptr(), od.data_ptr(), on.data_ptr(),
                    mode=H.MODE_COMPAT, ef=ef, stream=s)
    # a later clean search does not hide it (the word is sticky until read)
    g.set_option("vis_log2", 13)
    g.search_device(dq.data_ptr(), len(Q), Q.shape[1], 10, ok.data_ptr(), od.data_ptr(), on.data_ptr(),
                    mode=H.MODE_BEAM, ef=64, stream=s)
    with pytest.raises(H.HnswError, match="visited set overflow"):
        g.device_status()
    g.device_status()  # cleared
    # the clean device search is clean
    g.search_device(dq.data_ptr(), len(Q), Q.shape[1], k, ok.data_ptr(), od.data_ptr(), on.data_ptr(),
                    mode=H.MODE_COMPAT, ef=ef, stream=s)
    g.device_status()
    torch.cuda.synchronize()
    assert np.array_equal(on.cpu().numpy(), gn)
    assert np.array_equal(ok.cpu().numpy()[:, :k], gk)
    g.close()


@pytest.fixture(scope="module")
def wide(H, O):
    """an isotropic 32-dimensional set (no low-dimensional structure), where an
    ef-512 search meets thousands of nodes"""
    rng = np.random.default_rng(77)
    n, d = 100000, 32
    X = rng.normal(size=(n, d)).astype(np.float32)
    Q = rng.normal(size=(64, d)).astype(np.float32)
    g = H.Graph(M=12, Ml=0.25, EfSearch=64, Distance=_metric_fn(H, 1), Rng=5, build_mode=H.BUILD_BATCH,
                ef_construction=64, heuristic=2, m0=24)
    g.add_arrays(np.arange(n), X)
    o = O.Graph(metric=1, order=O.ORDER_DEV, M=12, M0=24, Ml=0.25, EfSearch=64)
    o.import_graph(**g.export())
    yield g, o, Q
    g.close()


def test_compact_visited_set(H, O, wide):
    """The compact set (16-bit entries, 8,192 ids in 16 KiB; option vis_compact,
    on by default when ids < 2^24) against the 32-bit set (5,120 ids in 20 KiB)
    at ef 512, where the 32-bit set fills: both equal the oracle (which never
    forgets), the compact set resets less and evaluates less."""
    g, o, Q = wide
    rk, rd, rn = o.search(Q, 10, mode=O.MODE_BEAM, ef=512)
    st = {}
    for c in (0, 1):
        g.set_option("vis_compact", c)
        g.reset_stats()
        gk, gd, gn = g.search_arrays(Q, 10, mode=H.MODE_BEAM, ef=512)
        st[c] = g.stats()
        _same_results(gk, gd, gn, rk, rd, rn)
    g.set_option("vis_compact", 1)
    print({c: (s["visited_resets"], s["search_dist_evals"]) for c, s in st.items()})
    assert st[0]["visited_resets"] >= len(Q), st
    assert st[1]["visited_resets"] < st[0]["visited_resets"], st
    assert st[1]["search_dist_evals"] < st[0]["search_dist_evals"], st
    # some queries fill the compact set too: its resets and the re-seeding after
    # them were part of the oracle comparison above
    assert st[1]["visited_resets"] > 0, st
