"""GPU: the north-star sharded search through the HIP engine.

Node-ID range shards (hnsw_amd.shard.shard_range), each an independent engine
handle over its key range; every query searched on every shard with
mhnsw_search_device; per-shard (dist, key) top-k merged on the GPU by
mhnsw_merge_topk_device.  Checked against:
  * exact mode: the single-index exact top-k (sharding must not change it);
  * beam mode: the merge (tests/test_distributed.merge_reference) of the
    oracle's beam search on each shard's graph;
and, across two processes (gloo world 2, both ranks on cuda:0), the packed
all-gather of hnsw_amd.shard.gather_topk between the engine and the merge.
"""
import os
import socket

import numpy as np
import pytest

from tests.test_distributed import merge_reference
from tests.test_gpu_parity import _clustered, _metric_fn, _same_results

pytestmark = pytest.mark.gpu


def _data(n, d, nq, seed):
    rng = np.random.default_rng(seed)
    return _clustered(rng, n, d), _clustered(rng, nq, d)


def _shards(H, X, S, metric, keys):
    from hnsw_amd.shard import shard_range

    out = []
    for s in range(S):
        lo, hi = shard_range(len(X), S, s)
        g = H.Graph(M=12, Ml=0.25, EfSearch=48, Distance=_metric_fn(H, metric), Rng=s, build_mode=H.BUILD_BATCH,
                    ef_construction=64, heuristic=2, m0=24)
        g.add_arrays(keys[lo:hi], X[lo:hi])
        out.append((g, lo, hi))
    return out


@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("S", [2, 3, 8])
def test_sharded_engine_search_merge(H, O, metric, S):
    torch = pytest.importorskip("torch")
    from hnsw_amd.shard import engine_local_search, merge_topk

    n, d, B, k = 9000, 64, 200, 10
    X, Q = _data(n, d, B, 5 + S + metric)
    keys = np.arange(n, dtype=np.int64) * 5 - 1000
    shards = _shards(H, X, S, metric, keys)
    dev = torch.device("cuda:0")
    dq = torch.from_numpy(Q).to(dev)
    full = H.Graph(M=12, Ml=0.25, EfSearch=48, Distance=_metric_fn(H, metric), Rng=9, build_mode=H.BUILD_FLAT)
    full.add_arrays(keys, X)
    fk, fd, fn = full.search_arrays(Q, k, mode=H.MODE_EXACT)
    for mode, ef in ((H.MODE_EXACT, 0), (H.MODE_BEAM, 48), (H.MODE_BEAM, 160)):
        lists = [engine_local_search(g, k, mode, ef)(dq) for g, _, _ in shards]
        ak = torch.stack([x[0] for x in lists])
        ad = torch.stack([x[1] for x in lists])
        an = torch.stack([x[2] for x in lists])
        for g, _, _ in shards:
            g.device_status()
        mk, md, mn = (x.cpu().numpy() for x in merge_topk(ak, ad, an, k))
        if mode == H.MODE_EXACT:
            _same_results(mk, md, mn, fk, fd, fn)
            continue
        # the same per-shard beam searches on the oracle, merged by the numpy restatement
        per = []
        for g, lo, hi in shards:
            o = O.Graph(metric=metric, order=O.ORDER_DEV, M=12, M0=24, Ml=0.25, EfSearch=48)
            o.import_graph(**g.export())
            per.append(o.search(Q, k, mode=O.MODE_BEAM, ef=ef))
        rk, rd, rn = (x.numpy() for x in merge_reference(np.stack([p[0] for p in per]), np.stack([p[1] for p in per]),
                                                          np.stack([p[2] for p in per]), k))
        _same_results(mk, md, mn, rk, rd, rn)
        # and the engine's per-shard lists are the oracle's
        for s, p in enumerate(per):
            _same_results(ak[s].cpu().numpy(), ad[s].cpu().numpy(), an[s].cpu().numpy(), *p)
        # sharded beam recall vs the exact top-k is at least that of the shards' lists alone
        rec = np.mean([len(set(mk[b, : mn[b]]) & set(fk[b, : fn[b]])) / k for b in range(B)])
        assert rec >= 0.9, rec
    for g, _, _ in shards:
        g.close()
    full.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_q):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import hnsw_amd as H
        from hnsw_amd.shard import engine_local_search, shard_range, sharded_search

        torch.cuda.set_device(0)
        n, d, B, k = 6000, 48, 128, 10
        X, Q = _data(n, d, B, 21)
        lo, hi = shard_range(n, world, rank)
        g = H.Graph(M=12, Ml=0.25, EfSearch=48, Distance=H.CosineDistance, Rng=rank, build_mode=H.BUILD_BATCH,
                    ef_construction=64, heuristic=2, m0=24)
        g.add_arrays(np.arange(lo, hi, dtype=np.int64), X[lo:hi])
        dq = torch.from_numpy(Q).cuda()
        res = {}
        for name, mode, ef in (("exact", H.MODE_EXACT, 0), ("beam", H.MODE_BEAM, 64)):
            mk, md, mn = sharded_search(engine_local_search(g, k, mode, ef), dq, k)
            g.device_status()
            local = engine_local_search(g, k, mode, ef)(dq)
            res[name] = tuple(x.cpu().numpy() for x in (mk, md, mn)) + tuple(x.cpu().numpy() for x in local)
        g.close()
        out_q.put((rank, res))
    finally:
        dist.barrier()
        dist.destroy_process_group()


def test_sharded_engine_gloo_world2(H, O):
    """two ranks (processes) on one GPU, gloo all-gather staged through the host"""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(2))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    n, d, B, k = 6000, 48, 128, 10
    X, Q = _data(n, d, B, 21)
    full = H.Graph(M=12, Ml=0.25, EfSearch=48, Distance=H.CosineDistance, build_mode=H.BUILD_FLAT)
    full.add_arrays(np.arange(n, dtype=np.int64), X)
    fk, fd, fn = full.search_arrays(Q, k, mode=H.MODE_EXACT)
    full.close()
    for name in ("exact", "beam"):
        r0, r1 = got[0][name], got[1][name]
        # both ranks hold the same merged answer
        for a, b in zip(r0[:3], r1[:3]):
            assert np.array_equal(a, b)
        # = the numpy merge of the two ranks' local lists
        rk, rd, rn = (x.numpy() for x in merge_reference(np.stack([r0[3], r1[3]]), np.stack([r0[4], r1[4]]),
                                                          np.stack([r0[5], r1[5]]), k))
        _same_results(r0[0], r0[1], r0[2], rk, rd, rn)
        if name == "exact":  # = the single-index exact top-k
            _same_results(r0[0], r0[1], r0[2], fk, fd, fn)


def test_config3_full_size(H, O):
    """BASELINE configs[3] at its stated size on one GPU: 10M x 768-d cosine in
    8 node-ID range shards of 1.25M rows, each built by the batched insert with
    the bench's graph recipe; every query searched on every shard and the
    per-shard top-k merged (the 8-GPU layout, each shard a separate handle).
    Sharded exact == the exact top-k of one flat index over all 10M rows,
    bitwise; sharded beam (ef 64) recall@10 >= 0.99 against it; the first and
    last shards' beam lists == the oracle's beam search (graph.go:1047-1110) on
    each exported shard graph for 512 queries (keys, counts, distance bits)."""
    torch = pytest.importorskip("torch")
    from bench import gen_vectors
    from hnsw_amd.shard import engine_local_search, merge_topk, shard_range

    S, n, d, B, k = 8, 10_000_000, 768, 4096, 10
    dev = torch.device("cuda:0")
    X = gen_vectors(n, d, 1234, 12, 1000, dev, "cosine")
    Q = gen_vectors(B, d, 9011, 12, 1000, dev, "cosine")
    keys = np.arange(n, dtype=np.int64)
    torch.cuda.synchronize()  # the handles read X on their own streams
    shards = []
    for s in range(S):
        lo, hi = shard_range(n, S, s)
        g = H.Graph(M=16, Ml=0.25, EfSearch=64, Distance=H.CosineDistance, Rng=1234 + s, build_mode=H.BUILD_BATCH,
                    m0=40, ef_construction=400, heuristic=2, keep_pruned=1, prune_alpha_pct=115)
        g.reserve(hi - lo, d)
        g.add_device(keys[lo:hi], X[lo:hi].contiguous().data_ptr(), hi - lo, d)
        shards.append(g)
        print(f"shard {s}: {hi - lo} rows built", flush=True)
    full = H.Graph(M=16, Ml=0.25, EfSearch=64, Distance=H.CosineDistance, build_mode=H.BUILD_FLAT, screen=0)
    full.reserve(n, d)
    full.add_device(keys, X.data_ptr(), n, d)
    del X
    fk, fd, fn = engine_local_search(full, k, H.MODE_EXACT, 0)(Q)
    full.device_status()
    fk, fd, fn = fk.cpu().numpy(), fd.cpu().numpy(), fn.cpu().numpy()
    full.close()
    res = {}
    for name, mode, ef in (("exact", H.MODE_EXACT, 0), ("beam", H.MODE_BEAM, 64)):
        lists = [engine_local_search(g, k, mode, ef)(Q) for g in shards]
        for g in shards:
            g.device_status()
        mk, md, mn = merge_topk(torch.stack([x[0] for x in lists]), torch.stack([x[1] for x in lists]),
                                torch.stack([x[2] for x in lists]), k)
        res[name] = (mk.cpu().numpy(), md.cpu().numpy(), mn.cpu().numpy())
        if mode == H.MODE_BEAM:
            from bench import host_threads

            Qh = Q[:512].cpu().numpy()
            for s in (0, S - 1):
                o = O.Graph(metric=O.COSINE, order=O.ORDER_DEV, M=16, M0=40, Ml=0.25, EfSearch=64)
                o.import_graph(**shards[s].export())
                want = o.search(Qh, k, mode=O.MODE_BEAM, ef=64, threads=max(1, min(64, host_threads())))
                del o
                _same_results(*(x[:512].cpu().numpy() for x in lists[s]), *want)
                print(f"shard {s}: 512 beam lists == oracle", flush=True)
    _same_results(*res["exact"], fk, fd, fn)
    mk, _, mn = res["beam"]
    rec = np.mean([len(set(mk[b, : mn[b]]) & set(fk[b, : fn[b]])) / k for b in range(B)])
    assert rec >= 0.99, rec
    for g in shards:
        g.close()
