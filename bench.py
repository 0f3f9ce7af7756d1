#!/usr/bin/env python3
"""Headline benchmark: queries/sec @ recall@10 on 1M x 768-d cosine
(BASELINE.json configs[1]: single MI355X, batched-query HIP search, ef=64, k=10).

A "step" = one batched layer-descent + layer-0 beam search of `--batch` query
vectors already resident in HBM, through the C ABI (mhnsw_search_device).

Multi-GPU (one process per GPU, torchrun).  Two layouts, both measured by
default (the headline `value` is the replica layout; the shard layout is the
`shard` object of the same JSON line):
  replica: every rank holds the full 1M-vector index and serves its own slice
      of the query stream; no data-path collective (per-GPU work fixed =>
      "scaling": "weak").
  shard (north_star): node-ID range sharding -- rank r owns keys
      [r*n, (r+1)*n) of one N*n-row dataset and its own sub-graph; every query
      is searched on every shard, the per-shard (dist, key) top-k are packed
      into one buffer, all-gathered in ONE collective over RCCL (xGMI) and
      merged on the GPU (mhnsw_merge_topk_device).  The index grows with the GPU
      count (BASELINE config 4: 10M over 8 GPUs), so shard QPS measures the
      capacity layout, not a throughput layout.
  --mode shard makes the shard layout the headline (and skips the replica leg).

Also reported: recall@10 against the exact (MFMA brute-force) path, build
throughput of the batched insert, the search kernel's roofline (HBM-bound;
algorithmic bytes from in-kernel distance-evaluation / expansion counters), and
the CPU restatement (oracle/, same algorithm, same graph) timed on a bounded
sample on the host.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import hnsw_amd as H  # noqa: E402

# revision of the search/build kernels the recorded PMC passes (profiles/*_pmc_*.json)
# were taken on; a pass recorded on another revision is not attached as `traffic`
KERNEL_REV = "r02-rowmajor-selection"
from hnsw_amd.shard import engine_local_search, shard_range, sharded_search  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--mode", choices=["replica", "shard"], default="replica",
                   help="headline layout; with replica the shard layout is measured too (--no-shard-leg skips it)")
    p.add_argument("--no-shard-leg", action="store_true")
    p.add_argument("--nbase", type=int, default=1_000_000, help="vectors per index (per shard in shard mode)")
    p.add_argument("--dim", type=int, default=768)
    p.add_argument("--batch", type=int, default=65536, help="queries per step per GPU")
    p.add_argument("--ef", type=int, default=64)
    p.add_argument("--k", type=int, default=10)
    p.add_argument("--metric", choices=["cosine", "euclidean"], default="cosine")
    p.add_argument("--M", type=int, default=16)
    p.add_argument("--M0", type=int, default=40)
    p.add_argument("--efc", type=int, default=400)
    p.add_argument("--keep-pruned", type=int, default=1)
    p.add_argument("--alpha", type=int, default=115, help="heuristic slack x100 (prune_alpha_pct; 100 = HNSW Alg. 4)")
    p.add_argument("--build-expand", type=int, default=2, choices=[1, 2],
                   help="entries expanded per step of the batched insert's layer searches")
    p.add_argument("--screen", type=int, default=1,
                   help="1: fp16 screening copy, 0: plain f32 evaluation of every candidate; same results")
    p.add_argument("--ef-sweep", default="32,48,64,72,80,96,128,256",
                   help="extra operating points (ef values) reported at N=1; '' disables")
    p.add_argument("--seed", type=int, default=1234)
    p.add_argument("--intrinsic", type=int, default=12)
    p.add_argument("--clusters", type=int, default=1000)
    p.add_argument("--gt-queries", type=int, default=4096, help="queries scored against exact top-k")
    p.add_argument("--cpu-seconds", type=float, default=20.0, help="CPU baseline time box (0 disables)")
    p.add_argument("--backend", default="nccl", help="nccl (= RCCL on ROCm) or gloo (rehearsal)")
    p.add_argument("--one-gpu", action="store_true", help="map every rank to cuda:0 (multi-rank rehearsal)")
    p.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "r02_pmc_search.json"))
    p.add_argument("--pmc-build-json", default=os.path.join(ROOT, "profiles", "r02_pmc_build.json"))
    return p.parse_args()


def gen_vectors(n, dim, seed, intrinsic, clusters, device, metric, offset=0):
    """Synthetic embeddings with low intrinsic dimension: a Gaussian mixture of
    `clusters` centres in R^intrinsic, mapped to R^dim by a fixed random linear
    map, plus isotropic noise; L2-normalised for cosine.  Rows [offset, offset+n)
    of the stream defined by `seed` (chunked so any slice is reproducible)."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    C = torch.randn(clusters, intrinsic, generator=g, device=device)
    A = torch.randn(intrinsic, dim, generator=g, device=device) / intrinsic ** 0.5
    out = torch.empty(n, dim, device=device)
    chunk = 1 << 16
    first, last = offset // chunk, (offset + n - 1) // chunk
    for c in range(first, last + 1):
        gc = torch.Generator(device=device)
        gc.manual_seed(seed * 1_000_003 + c + 1)
        cid = torch.randint(0, clusters, (chunk,), generator=gc, device=device)
        z = C[cid] + 0.5 * torch.randn(chunk, intrinsic, generator=gc, device=device)
        x = z @ A + 0.05 * torch.randn(chunk, dim, generator=gc, device=device)
        if metric == "cosine":
            x = x / x.norm(dim=1, keepdim=True)
        lo, hi = max(offset, c * chunk), min(offset + n, (c + 1) * chunk)
        out[lo - offset:hi - offset] = x[lo - c * chunk:hi - c * chunk]
    return out.contiguous()


class Searcher:
    def __init__(self, g, B, k, dim, device):
        self.g, self.B, self.k, self.dim = g, B, k, dim
        self.keys = torch.empty(B, k, dtype=torch.int64, device=device)
        self.dist = torch.empty(B, k, dtype=torch.float32, device=device)
        self.n = torch.empty(B, dtype=torch.int32, device=device)

    def run(self, q, mode, ef):
        s = torch.cuda.current_stream().cuda_stream
        self.g.search_device(q.data_ptr(), q.shape[0], self.dim, self.k, self.keys.data_ptr(), self.dist.data_ptr(),
                             self.n.data_ptr(), mode=mode, ef=ef, stream=s)
        return self.keys, self.dist, self.n


def recall_at_k(res, n, truth, tn, k):
    res, n, truth, tn = (x.cpu().numpy() for x in (res, n, truth, tn))
    tot = 0.0
    for b in range(res.shape[0]):
        t = set(truth[b, : tn[b]].tolist())
        tot += len(set(res[b, : n[b]].tolist()) & t) / max(1, min(k, len(t)))
    return tot / res.shape[0]


def cpu_baseline(g, queries_np, k, ef, metric, seconds):
    """The CPU restatement (oracle/, test infrastructure) timed on this host on a
    bounded sample: same graph, same beam algorithm; plus the reference's
    compat Search() semantics.  Single thread, sequential queries
    (= BatchSearch's loop, graph.go:1075)."""
    import oracle as O  # checker / baseline only

    ex = g.export()
    o = O.Graph(metric=O.COSINE if metric == "cosine" else O.EUCLIDEAN, order=O.ORDER_REF, M=g.M,
                M0=g.get_option("m0"), Ml=g.Ml, EfSearch=ef)
    o.import_graph(**ex)
    del ex
    out = {}
    threads = min(16, os.cpu_count() or 1)  # the GPU box's CPU share is 16
    for name, mode, nt, frac in (("beam", O.MODE_BEAM, 1, 0.4), ("compat", O.MODE_COMPAT, 1, 0.3),
                                 ("beam_mt", O.MODE_BEAM, threads, 0.3)):
        chunk = 32 * nt
        done, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < seconds * frac and done < len(queries_np):
            o.search(queries_np[done:done + chunk], k, mode=mode, ef=ef, threads=nt)
            done += min(chunk, len(queries_np) - done)
        out[name] = (done / (time.perf_counter() - t0), done, nt)
    return out


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.one_gpu:
        local = 0
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(a.backend)
    metric = H.CosineDistance if a.metric == "cosine" else H.EuclideanDistance

    # ---- replica index: rows [0, nbase) on every rank ---------------------------
    shard_only = a.mode == "shard"

    sweep = None

    def build(off, rng_seed):
        nonlocal sweep
        X = gen_vectors(a.nbase, a.dim, a.seed, a.intrinsic, a.clusters, device, a.metric, offset=off)
        g = H.Graph(M=a.M, Ml=0.25, EfSearch=a.ef, Distance=metric, Rng=rng_seed, build_mode=H.BUILD_BATCH,
                    m0=a.M0, ef_construction=a.efc, heuristic=2, keep_pruned=a.keep_pruned, prune_alpha_pct=a.alpha,
                    build_expand=a.build_expand,
                    screen=a.screen, time_build=1)
        g.reserve(a.nbase, a.dim)
        keys = np.arange(off, off + a.nbase, dtype=np.int64)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.add_device(keys, X.data_ptr(), a.nbase, a.dim)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if sweep is None and rank == 0:
            sweep = sweep_bench(X)
        del X
        return g, dt, g.stats()

    def sweep_bench(X, reps=10):
        """K1 microbench: one query against every row, mhnsw_distance_device;
        HBM-bound at n*d*4 bytes per sweep, HIP events on the launch stream."""
        out = torch.empty(X.shape[0], dtype=torch.float32, device=device)
        q = X[12345].clone()
        s = torch.cuda.current_stream()
        H.sweep_device(metric.metric, q.data_ptr(), X.data_ptr(), X.shape[0], a.dim, out.data_ptr(), s.cuda_stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            H.sweep_device(metric.metric, q.data_ptr(), X.data_ptr(), X.shape[0], a.dim, out.data_ptr(),
                           s.cuda_stream)
        e1.record(s)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        byts = X.shape[0] * a.dim * 4
        return {"kernel": "k_sweep_raw4", "rows": X.shape[0], "dim": a.dim, "ms": round(ms, 4),
                "alg_bytes": byts, "achieved_GBps": round(byts / ms / 1e6, 1),
                "frac": round(byts / ms / 1e6 / HBM_PEAK_GBS, 4),
                "self_distance_zero": bool(abs(float(out[12345])) <= 1e-6)}

    qseed = a.seed + 7_777
    ngt = min(a.gt_queries, a.batch)

    def timed_steps(step, g):
        for _ in range(a.warmup):
            step()
        g.reset_stats()
        kernel_ms = []
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
            kernel_ms.append(g.last_kernel_ms())
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        g.device_status()  # kernel-side errors of the asynchronous searches
        tt = torch.tensor([elapsed], dtype=torch.float64, device=device)
        if world > 1:
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        return tt.item(), kernel_ms, g.stats()

    def mean_over_ranks(x):
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=device)
        dist.all_reduce(t)
        return t.item() / world

    g = None
    if not shard_only:
        g, build_s, bstats = build(0, a.seed)
        Q = gen_vectors(a.batch, a.dim, qseed, a.intrinsic, a.clusters, device, a.metric, offset=rank * a.batch)
        S = Searcher(g, a.batch, a.k, a.dim, device)

        def step():
            return S.run(Q, H.MODE_BEAM, a.ef)

        # recall vs exact on the same index
        res_k, _, res_n = (x.clone() for x in step())
        G = Searcher(g, ngt, a.k, a.dim, device)
        tk, td, tn = G.run(Q[:ngt], H.MODE_EXACT, 0)
        torch.cuda.synchronize()
        recall = mean_over_ranks(recall_at_k(res_k[:ngt], res_n[:ngt], tk, tn, a.k))
        elapsed, kernel_ms, st = timed_steps(step, g)

    # ---- shard layout: rank r owns rows [r*nbase, (r+1)*nbase) of one dataset --------
    shard_out = None
    if shard_only or not a.no_shard_leg:
        lo, _ = shard_range(a.nbase * world, world, rank)
        if g is not None and lo == 0:
            gs, sbuild_s, sbstats = g, build_s, bstats  # rank 0's shard is the replica index
        else:
            gs, sbuild_s, sbstats = build(lo, a.seed + rank)
        Qs = gen_vectors(a.batch, a.dim, qseed, a.intrinsic, a.clusters, device, a.metric)  # same on every rank

        def sstep():
            return sharded_search(engine_local_search(gs, a.k, H.MODE_BEAM, a.ef), Qs, a.k)

        sk, _, sn = (x.clone() for x in sstep())
        ek, ed, en = sharded_search(engine_local_search(gs, a.k, H.MODE_EXACT, 0), Qs[:ngt], a.k)
        torch.cuda.synchronize()
        srecall = mean_over_ranks(recall_at_k(sk[:ngt], sn[:ngt], ek, en, a.k))
        s_el, s_kms, s_st = timed_steps(sstep, gs)
        skms = float(np.mean(s_kms))
        shard_out = {
            "value": round(a.batch * a.steps / s_el, 1), "unit": "queries/s",
            "ms_per_step": round(s_el / a.steps * 1e3, 3), "recall_at_10": round(srecall, 4),
            "n_base_total": a.nbase * world, "shards": world, "rows_per_shard": a.nbase,
            "queries_per_step": a.batch, "search_kernel_ms": round(skms, 4),
            "exchange": ("none (one shard)" if world == 1 else
                         f"one all-gather of {a.batch * (12 * a.k + 4)} B per rank ({a.backend}), k_merge on the GPU"),
            "recall_reference": "sharded exact search (per-shard MFMA exact + the same gather + merge)",
            "build_inserts_per_s_per_rank": round(a.nbase / sbuild_s, 1),
        }
        if shard_only:
            g, build_s, bstats, recall, elapsed, kernel_ms, st = gs, sbuild_s, sbstats, srecall, s_el, s_kms, s_st
            Q, S = Qs, Searcher(gs, a.batch, a.k, a.dim, device)
            tk, tn = ek, en

    def build_roofline(bs, secs):
        """Batched insert (configs[2] kernel family, here on the bench index): the
        search kernels' algorithmic bytes -- f32 rows (4d + 4: row + norm) for every
        f32 evaluation and neighbour-selection row, fp16 rows (2d) for every screened
        candidate, one layer-0 adjacency row per expansion, the new row and its
        adjacency/proposal writes -- over their device time (HIP events)."""
        F, Sc, Xp = bs["build_f32_rows"], bs["build_screened"], bs["build_expansions"]
        aux = 8 if a.metric == "euclidean" else 0
        byts = F * (4 * a.dim + 4) + Sc * (2 * a.dim + aux) + Xp * 4 * (a.M0 + 1) + a.nbase * (4 * a.dim + 16 * a.M0)
        us = bs["build_search_us"]
        gbs = byts / (us * 1e-6) / 1e9 if us > 0 else None
        # HBM bytes of k_batch_search from a separate rocprofv3 --pmc pass of this
        # same configuration (tools/profile_round.sh), when one is recorded
        traffic = None
        try:
            pm = json.load(open(a.pmc_build_json))
            want = dict(n=a.nbase, dim=a.dim, efc=a.efc, m0=a.M0, keep_pruned=a.keep_pruned, alpha=a.alpha,
                        screen=a.screen, rev=KERNEL_REV)
            if all(pm.get(k) == v for k, v in want.items()):
                traffic = pm.get("hbm_bytes_total")
        except (OSError, ValueError):
            traffic = None
        return {"inserts_per_s": round(a.nbase / secs, 1), "seconds": round(secs, 2),
                "dist_evals_per_insert": round(bs["build_dist_evals"] / a.nbase, 1),
                "f32_rows_per_insert": round(F / a.nbase, 1), "screened_per_insert": round(Sc / a.nbase, 1),
                "expansions_per_insert": round(Xp / a.nbase, 1), "dropped_proposals": bs["dropped_proposals"],
                "roofline": {"bound": "hbm", "kernel": "k_batch_search + k_batch_descend",
                             "kernel_ms_total": round(us / 1e3, 2), "alg_bytes": int(byts),
                             "achieved": round(gbs, 1) if gbs else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": round(gbs / HBM_PEAK_GBS, 4) if gbs else None,
                             "traffic": traffic, "traffic_kernel": "k_batch_search"}}

    shard = shard_only
    queries_done = a.batch * a.steps * (1 if shard else world)
    qps = queries_done / elapsed

    # roofline of the search kernel (per launch = one step on this GPU)
    cap0 = a.M0 + 1

    def alg_bytes_of(stats, launches):
        # f32 row + norm per f32 evaluation, fp16 row per screened candidate,
        # one adjacency row per expansion, the query
        E = stats["search_dist_evals"] / launches
        Sc = stats["search_screened"] / launches
        F = stats["search_f32_evals"] / launches
        Xp = stats["search_expansions"] / launches
        aux = 8 if a.metric == "euclidean" else 0  # L2 screening reads {unscale, |x|} per row
        return (F * (4 * a.dim + 4) + Sc * (2 * a.dim + aux) + Xp * 4 * cap0
                + a.batch * 4 * a.dim, E, Xp, Sc, F)

    alg_bytes, E, Xp, Sc, F = alg_bytes_of(st, a.steps)
    kms = float(np.mean(kernel_ms))
    achieved = alg_bytes / (kms * 1e-3) / 1e9

    # other operating points of the same graph (N=1 only): recall / QPS per ef
    points = []
    if world == 1 and a.ef_sweep:
        for ef in [int(x) for x in a.ef_sweep.split(",") if x]:
            kk, _, nn = (x.clone() for x in S.run(Q, H.MODE_BEAM, ef))
            r = recall_at_k(kk[:ngt], nn[:ngt], tk, tn, a.k)
            g.reset_stats()
            ms = []
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for _ in range(3):
                S.run(Q, H.MODE_BEAM, ef)
                ms.append(g.last_kernel_ms())
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t1) / 3
            ab, e_, _, _, _ = alg_bytes_of(g.stats(), 3)
            km = float(np.mean(ms))
            points.append({"ef": ef, "recall_at_10": round(r, 4), "qps": round(a.batch / dt, 1),
                           "kernel_ms": round(km, 4), "dist_evals_per_query": round(e_ / a.batch, 1),
                           "roofline_frac": round(ab / (km * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)})
    at99 = next((p for p in points if p["recall_at_10"] >= 0.99), None)
    traffic = None
    if os.path.exists(a.pmc_json):
        try:
            pm = json.load(open(a.pmc_json))
            want = dict(n=a.nbase, dim=a.dim, batch=a.batch, ef=a.ef, efc=a.efc, m0=a.M0, keep_pruned=a.keep_pruned,
                        alpha=a.alpha, screen=a.screen, rev=KERNEL_REV)
            if all(pm.get(k) == v for k, v in want.items()):
                traffic = pm.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    out = {
        "metric": "queries/sec @ recall@10, 1M×768-d cosine; 1/2/4/8-GPU scaling",
        "value": round(qps, 1),
        "unit": "queries/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(elapsed / a.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": (f"synthetic: {a.clusters}-centre Gaussian mixture in R^{a.intrinsic} mapped to R^{a.dim} by a "
                 f"random linear map + N(0,0.05^2) noise, L2-normalised; seed {a.seed}; queries from the same "
                 f"distribution (seed {qseed})"),
        "config": {
            "workload": (f"{a.nbase // 1000}k x {a.dim}-d {a.metric}, batched beam search ef={a.ef} k={a.k}, "
                         f"{a.batch} queries/step/GPU (BASELINE configs[1])") if not shard else
                        (f"{world} node-ID range shards of {a.nbase // 1000}k x {a.dim}-d {a.metric}, every query on "
                         f"every shard, beam ef={a.ef} k={a.k}, {a.batch} queries/step (BASELINE configs[3] layout)"),
            "n_base": a.nbase * (world if shard else 1), "dim": a.dim, "batch_per_gpu": a.batch, "ef": a.ef,
            "k": a.k, "M": a.M, "M0": a.M0, "ef_construction": a.efc, "keep_pruned": a.keep_pruned,
            "prune_alpha": a.alpha / 100,
            "screen": (("fp16"
                        + " row copy rejects candidates whose f32 distance provably exceeds the list's worst; "
                        "every reported distance is f32, results identical to screen=0") if a.screen else "off"),
            "parallelism": f"{'shard' if shard else 'replica'}{world}",
        },
        "recall_at_10": round(recall, 4),
        "parity": ("results bit-identical to oracle/, a C restatement of graph.go/distance.go (the Go toolchain "
                   "is absent, so parity is to the restatement, pinned by the reference's own test vectors: "
                   "tests/golden/reference_goldens.json); checked by pytest -m gpu, not inside this run"),
        "roofline": {
            "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "kernel": "k_search_beam", "kernel_ms": round(kms, 4),
            "alg_bytes_per_launch": int(alg_bytes),
            "dist_evals_per_query": round(E / a.batch, 1), "expansions_per_query": round(Xp / a.batch, 1),
            "screened_per_query": round(Sc / a.batch, 1), "f32_evals_per_query": round(F / a.batch, 1),
            "screen_margin": (g.get_option("screen_err_ppb") * 1e-9) if (g is not None and a.screen) else None,
        },
        "build": build_roofline(bstats, build_s),
        "sweep": sweep,
        "cpu_baseline": None,
        "operating_points": points,
        "at_recall_0.99": at99,
    }
    if shard_out is not None and not shard_only:
        out["shard"] = shard_out
    if rank == 0 and world == 1 and a.cpu_seconds > 0:
        qn = Q[: min(a.batch, 4096)].cpu().numpy()
        cb = cpu_baseline(g, qn, a.k, a.ef, a.metric, a.cpu_seconds)
        out["cpu_baseline"] = {
            "value": round(cb["beam"][0], 2), "unit": "queries/s", "cores": 1, "kind": "port",
            "sample": f"{cb['beam'][1]} of the same queries, same 1M graph, oracle beam search (ORDER_REF "
                      f"sequential fp32), single thread, ~{a.cpu_seconds * 0.4:.0f}s time box",
            "compat_search_qps": round(cb["compat"][0], 2), "compat_sample": cb["compat"][1],
            "beam_mt_qps": round(cb["beam_mt"][0], 2), "beam_mt_threads": cb["beam_mt"][2],
            "beam_mt_sample": cb["beam_mt"][1], "host_cpus": os.cpu_count(),
        }
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
