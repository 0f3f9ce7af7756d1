"""CPU, world_size 2 over gloo: node-ID range sharding + all-gather of per-shard
top-k + merge by (distance, key) reproduces the single-index exact top-k.
The per-shard searcher here is the CPU restatement (oracle/, exact mode) and
the merge is a numpy restatement of k_merge; the GPU merge kernel itself is
checked in tests/test_gpu_parity.py::test_merge_topk_device."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def merge_order(d, key):
    """k_merge's total order: distance (-0 == +0, NaN after +inf), then key."""
    d = float(d)
    return (d != d, 0.0 if d != d else d, int(key))


def merge_reference(ak, ad, an, k):
    """numpy restatement of k_merge: best k of all shard entries by (dist, key)."""
    S, B = an.shape
    ok = np.full((B, k), -1, np.int64)
    od = np.full((B, k), np.inf, np.float32)
    on = np.zeros(B, np.int32)
    for b in range(B):
        ents = [(ad[s, b, j], ak[s, b, j]) for s in range(S) for j in range(int(an[s, b]))]
        cand = sorted(ents, key=lambda e: merge_order(*e))[:k]
        on[b] = len(cand)
        for j, (d, key) in enumerate(cand):
            ok[b, j], od[b, j] = key, d
    return torch.from_numpy(ok), torch.from_numpy(od), torch.from_numpy(on)


def _worker(rank, world, port, n_total, dim, k, out_q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle as O
    from hnsw_amd.shard import shard_range, sharded_search

    rng = np.random.default_rng(0)
    X = rng.uniform(-1, 1, (n_total, dim)).astype(np.float32)
    Q = rng.uniform(-1, 1, (40, dim)).astype(np.float32)
    lo, hi = shard_range(n_total, world, rank)
    g = O.Graph(metric=O.COSINE, order=O.ORDER_DEV, M=8, Ml=0.25, EfSearch=20, seed=rank)
    g.add(np.arange(lo, hi), X[lo:hi], g.preview_levels(hi - lo))

    def local(qs):
        kk, dd, nn = g.search(qs.numpy(), k, mode=O.MODE_EXACT)
        return torch.from_numpy(kk), torch.from_numpy(dd), torch.from_numpy(nn)

    mk, md, mn = sharded_search(local, torch.from_numpy(Q), k,
                                merge=lambda a, b, c, kk: merge_reference(a.numpy(), b.numpy(), c.numpy(), kk))
    if rank == 0:
        full = O.Graph(metric=O.COSINE, order=O.ORDER_DEV, M=8, Ml=0.25, EfSearch=20)
        full.add(np.arange(n_total), X, full.preview_levels(n_total))
        fk, fd, fn = full.search(Q, k, mode=O.MODE_EXACT)
        out_q.put((mk.numpy(), md.numpy(), mn.numpy(), fk, fd, fn))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_exact_equals_single_index(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 3001, 24, 10, q)) for r in range(world)]
    for p in procs:
        p.start()
    mk, md, mn, fk, fd, fn = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert np.array_equal(mn, fn)
    assert np.array_equal(mk, fk)
    assert np.array_equal(md.view(np.uint32), fd.view(np.uint32))


def test_shard_ranges_partition():
    from hnsw_amd.shard import shard_range

    for n in (0, 1, 7, 10_000_000, 10_000_003):
        for w in (1, 2, 3, 8):
            rs = [shard_range(n, w, r) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
            assert max(h - l for l, h in rs) - min(h - l for l, h in rs) <= 1


def test_merge_reference_properties():
    rng = np.random.default_rng(3)
    S, B, k = 3, 50, 10
    ad = np.sort(rng.uniform(0, 1, (S, B, k)).astype(np.float32), axis=2)
    ak = rng.permutation(S * B * k).reshape(S, B, k).astype(np.int64)
    an = rng.integers(0, k + 1, (S, B)).astype(np.int32)
    ok, od, on = merge_reference(ak, ad, an, k)
    for b in range(B):
        assert on[b] == min(k, an[:, b].sum())
        d = od[b, : on[b]].numpy()
        assert np.all(d[:-1] <= d[1:])
