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
KERNEL_REV = "r06"
from hnsw_amd.shard import engine_local_search, gather_topk, merge_topk, shard_range, sharded_search  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--mode", choices=["replica", "shard"], default="replica",
                   help="headline layout; with replica the shard layout is measured too (--no-shard-leg skips it)")
    p.add_argument("--no-shard-leg", action="store_true")
    p.add_argument("--nbase", type=int, default=1_000_000, help="vectors of the replica index")
    p.add_argument("--total-rows", type=int, default=10_000_000,
                   help="rows of the sharded index over all ranks (BASELINE configs[3]: 10M, 1.25M per rank at 8)")
    p.add_argument("--configs", default="0,2,4,h",
                   help="secondary BASELINE configs measured at N=1 (configs[0] reference shape, [2] L2 build, "
                        "[4] exact, h harder data: latent 32 at ef up to 512); '' disables")
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
    p.add_argument("--batch-ratio", type=int, default=20,
                   help="batched insert: each batch holds this %% of the rows already in the index (batch_ratio_pct; "
                        "the engine default is 5, kept for incremental adds, include/mhnsw.h): fewer latency-bound small launches early on, recall@10 0.9904 vs "
                        "0.9909 at ef 64 on the bench index (profiles/r04_build_schedule.txt)")
    p.add_argument("--build-expand", type=int, default=4, choices=[1, 2, 3, 4],
                   help="entries expanded per step of the batched insert's layer searches (the engine default "
                        "since round 6; 4 builds the bench index 5.8 %% faster than 2 at the same recall@10, "
                        "0.9814 / 0.9904 at ef 48 / 64, profiles/r05_build_expand.txt)")
    p.add_argument("--upper-efc", type=int, default=128,
                   help="batched insert: candidate list of the layers above 0 (upper_efc; 0 = efConstruction): 128 "
                        "builds the bench index 22 %% faster at recall@10 0.9903 / 0.9814 at ef 64 / 48 "
                        "(0.9904 / 0.9814 with 0; profiles/r06_upper_efc.txt)")
    p.add_argument("--search-expand", type=int, default=1, choices=[1, 2, 4],
                   help="entries expanded per layer-0 step of the headline beam search (search_expand; 1 = the "
                        "standard search)")
    p.add_argument("--harder-build-expand", type=int, default=4, choices=[1, 2, 3, 4],
                   help="build_expand of the harder-data graph (configs 'h')")
    p.add_argument("--harder-upper-efc", type=int, default=256,
                   help="upper_efc of the harder-data graph: 256 builds it 17 %% faster at the same recall@10 "
                        "(0.9910 at ef 512; 128: 0.9909), profiles/r06_upper_efc.txt")
    p.add_argument("--emulate-shards", type=int, default=8,
                   help="N=1 only: build --total-rows as this many node-ID range shards (one handle each) on the one "
                        "GPU, search every shard and merge, and project the N-GPU rate at equal recall (0 disables)")
    p.add_argument("--screen", type=int, default=1,
                   help="1: fp16 screening copy, 0: plain f32 evaluation of every candidate; same results")
    p.add_argument("--ef-sweep", default="32,48,64,72,80,96,128,256",
                   help="extra operating points (ef values) reported at N=1; '' disables")
    p.add_argument("--shard-ef-sweep", default="16,24,32,40,48,64,96,128,192,256",
                   help="operating points of the shard layout (ef values; recall vs the sharded exact path); '' disables")
    p.add_argument("--batch-sweep", default="1,1024,10000",
                   help="query batch sizes re-measured at ef --ef on the same graph at N=1 (SURVEY 8(d) C2); '' disables")
    p.add_argument("--seed", type=int, default=1234)
    p.add_argument("--intrinsic", type=int, default=12)
    p.add_argument("--clusters", type=int, default=1000)
    p.add_argument("--gt-queries", type=int, default=4096, help="queries scored against exact top-k")
    p.add_argument("--cpu-seconds", type=float, default=20.0, help="CPU baseline time box (0 disables)")
    p.add_argument("--backend", default="nccl", help="nccl (= RCCL on ROCm) or gloo (rehearsal)")
    p.add_argument("--one-gpu", action="store_true", help="map every rank to cuda:0 (multi-rank rehearsal)")
    p.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "r06_pmc_search.json"))
    p.add_argument("--pmc-build-json", default=os.path.join(ROOT, "profiles", "r06_pmc_build.json"))
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


def host_threads():
    """CPUs this process can use: the affinity mask (nproc), capped by the
    cgroup's CPU quota when one is set (a container's share of a large host)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            parts = open(path).read().split()
            if path.endswith("cpu.max") and parts[0] != "max":
                n = min(n, max(1, int(int(parts[0]) / int(parts[1]))))
            elif path.endswith("quota_us") and int(parts[0]) > 0:
                period = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
                n = min(n, max(1, int(parts[0]) // period))
        except (OSError, ValueError, IndexError):
            continue
    return n


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def build_roofline(bs, secs, n, dim, m0, metric, traffic=None):
    """Batched insert: the insert kernels' algorithmic bytes -- f32 rows (4d + 4:
    row + norm) for every f32 evaluation and neighbour-selection row (the layer
    searches', their selection's and, since round 5, the commit's overflow
    pruning), fp16 rows
    (2d, + 8 for L2's {unscale, |x|}) for every screened candidate, one layer-0
    adjacency row per expansion, the new row and its adjacency/proposal writes --
    over the device time of every insert kernel (k_batch_descend, k_batch_search
    and k_batch_commit; HIP events around each layer's launches).  `wall_frac`
    puts the same bytes over the whole Add call's wall time."""
    F, Sc, Xp = bs["build_f32_rows"], bs["build_screened"], bs["build_expansions"]
    aux = 8 if metric == "euclidean" else 0
    byts = F * (4 * dim + 4) + Sc * (2 * dim + aux) + Xp * 4 * (m0 + 1) + n * (4 * dim + 16 * m0)
    us = bs["build_search_us"]
    gbs = byts / (us * 1e-6) / 1e9 if us > 0 else None
    return {"inserts_per_s": round(n / secs, 1), "seconds": round(secs, 2),
            "dist_evals_per_insert": round(bs["build_dist_evals"] / n, 1),
            "f32_rows_per_insert": round(F / n, 1), "screened_per_insert": round(Sc / n, 1),
            "expansions_per_insert": round(Xp / n, 1), "dropped_proposals": bs["dropped_proposals"],
            "roofline": {"bound": "hbm", "kernel": "k_batch_descend + k_batch_search + k_batch_commit",
                         "kernel_ms_total": round(us / 1e3, 2), "alg_bytes": int(byts),
                         "achieved": round(gbs, 1) if gbs else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(gbs / HBM_PEAK_GBS, 4) if gbs else None,
                         "wall_frac": round(byts / secs / 1e9 / HBM_PEAK_GBS, 4),
                         "traffic": traffic}}


def list_checksum(keys, dists, n):
    """order-sensitive int64 checksum of a batch of result lists (keys, distance
    bits, counts): equal on every rank when every rank merged the same lists"""
    B, k = keys.shape
    m = torch.arange(k, device=keys.device)[None, :] < n[:, None].long()
    kk = torch.where(m, keys, torch.full_like(keys, -1))
    db = torch.where(m, dists.contiguous().view(torch.int32).long(), torch.zeros_like(keys))
    w = torch.arange(1, B * k + 1, device=keys.device, dtype=torch.int64).view(B, k) * 0x9E3779B1 + 1
    return int(((kk * w) ^ (db * 0x2545F491)).sum().item() + int(n.long().sum().item()))


def timed(fn, reps=1):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        r = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps, r


def config0(device, seconds):
    """BASELINE configs[0], the reference's own CPU benchmark shape
    (graph_benchmark_test.go:50-89): 10k x 128 U[-1,1) cosine, M 16, Ml 0.25,
    EfSearch 20, k 10, 1000 queries -- with the reference's semantics end to end
    (compat Add and compat Search, graph.go:437-625) on the GPU, and the same
    Search restated in C (oracle/) on the host's cores on the same graph."""
    import oracle as O  # CPU baseline only

    n, d, nq, k = 10_000, 128, 1000, 10
    rng = np.random.default_rng(42)
    X = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    Qh = rng.uniform(-1, 1, (nq, d)).astype(np.float32)
    g = H.Graph(M=16, Ml=0.25, EfSearch=20, Distance=H.CosineDistance, Rng=42)  # compat build (reference Add)
    lv = g.preview_levels(n)  # the levels the engine's seed-42 stream gives (injected into the oracle)
    bt, _ = timed(lambda: g.add_arrays(np.arange(n), X))
    Q = torch.from_numpy(Qh).to(device)
    S = Searcher(g, nq, k, d, device)
    S.run(Q, H.MODE_COMPAT, 20)
    st, (ck, cd, cn) = timed(lambda: S.run(Q, H.MODE_COMPAT, 20), reps=20)
    g.device_status()
    ck, cd, cn = ck.clone(), cd.clone(), cn.clone()
    tk, _, tn = (x.clone() for x in Searcher(g, nq, k, d, device).run(Q, H.MODE_EXACT, 0))
    rec = recall_at_k(ck, cn, tk, tn, k)
    # the reference's Add (graph.go:437-531) in the reference's arithmetic (ORDER_REF),
    # the same levels, the whole 10k walk -- timed as the CPU baseline and compared
    ob = O.Graph(metric=O.COSINE, order=O.ORDER_REF, M=16, Ml=0.25, EfSearch=20)
    cbt, _ = timed(lambda: ob.add(np.arange(n), X, lv))
    from oracle.parity import compare_lists, same_graph

    graph_same = same_graph(g.export(), ob.export())
    par = compare_lists(tuple(x.cpu().numpy() for x in (ck, cd, cn)), ob.search(Qh, k, mode=O.MODE_COMPAT), k,
                        truth=(tk.cpu().numpy(), tn.cpu().numpy()))
    cpu = {}
    for name, nt in (("1_thread", 1), ("all_threads", host_threads())):
        chunk = max(nq, 64 * nt)
        done, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < seconds / 4:
            ob.search(Qh[np.arange(done, done + chunk) % nq], k, mode=O.MODE_COMPAT, threads=nt)
            done += chunk
        cpu[name] = round(done / (time.perf_counter() - t0), 1)
    g.close()
    return {"workload": "10k x 128-d U[-1,1) cosine, M=16 Ml=0.25 EfSearch=20, k=10, 1000 queries (reference "
                        "semantics: compat Add + compat Search)",
            "gpu_compat_add_inserts_per_s": round(n / bt, 1), "gpu_compat_search_qps": round(nq / st, 1),
            "recall_at_10_compat": round(rec, 4),
            "cpu_compat_search_qps": cpu["1_thread"], "cpu_compat_search_qps_all_threads": cpu["all_threads"],
            "cpu_threads": host_threads(), "cpu_model": cpu_model(),
            "cpu_compat_add_inserts_per_s": round(n / cbt, 1), "cpu_compat_add_sample": n,
            "cpu_kind": "port (oracle/: C restatement of graph.go, ORDER_REF sequential fp32; the Go toolchain is absent)",
            "parity_vs_order_ref": dict(par, graph_identical=bool(graph_same),
                                        what="GPU compat build + compat Search vs the oracle's Add + Search in "
                                             "ORDER_REF from the same levels (a = GPU, b = ORDER_REF)")}


def config2(device, build_expand=4, upper_efc=32, pmc_json=os.path.join(ROOT, "profiles", "r06_pmc_config2.json")):
    """BASELINE configs[2]: 1M x 768 Euclidean, the batched insert at SURVEY
    8(d) C3's efConstruction = EfSearch = 64 (graph.go:500), M 16; recall@10 of
    the built graph at ef 64 against the exact path."""
    n, d = 1_000_000, 768
    X = gen_vectors(n, d, 77, 12, 1000, device, "euclidean")
    Q = gen_vectors(4096, d, 78, 12, 1000, device, "euclidean")
    g = H.Graph(M=16, Ml=0.25, EfSearch=64, Distance=H.EuclideanDistance, Rng=5, build_mode=H.BUILD_BATCH,
                m0=48, ef_construction=64, heuristic=2, batch_ratio_pct=20, build_expand=build_expand,
                upper_efc=upper_efc, time_build=1)
    g.reserve(n, d)
    bt, _ = timed(lambda: g.add_device(np.arange(n), X.data_ptr(), n, d))
    bs = g.stats()
    del X
    tk, _, tn = (x.clone() for x in Searcher(g, 4096, 10, d, device).run(Q, H.MODE_EXACT, 0))
    k_, _, n_ = Searcher(g, 4096, 10, d, device).run(Q, H.MODE_BEAM, 64)
    rec = recall_at_k(k_, n_, tk, tn, 10)
    g.close()
    out = {"workload": f"1M x 768-d Euclidean batched insert, M=16 M0=48 efConstruction=64 (SURVEY 8(d) C3), "
                       f"batches of 20 % of the index, build_expand {build_expand}, upper_efc {upper_efc} "
                       f"(recall@10 0.9977 at ef 64 with 0, 32 and 16: profiles/r06_config2_sched.txt)"}
    traffic = None  # the insert kernels' HBM bytes from the PMC passes of this build (tools/profile_round.sh)
    try:
        pm = json.load(open(pmc_json)) if pmc_json else {}
        if all(pm.get(k) == v for k, v in dict(n=n, dim=d, efc=64, m0=48, build_expand=build_expand,
                                                upper_efc=upper_efc, batch_ratio=20, rev=KERNEL_REV).items()):
            traffic = pm.get("hbm_bytes_total")
    except (OSError, ValueError):
        pass
    out.update(build_roofline(bs, bt, n, d, 48, "euclidean", traffic))
    out["recall_at_10_ef64"] = round(rec, 4)
    return out


def config4(device, steps=10):
    """BASELINE configs[4]: 1M x 1536 cosine, batch 1024, the exact path (fp16
    MFMA scores with the fused preselection, canonical re-rank, certificate)."""
    n, d, B = 1_000_000, 1536, 1024
    X = gen_vectors(n, d, 55, 12, 1000, device, "cosine")
    Q = gen_vectors(B, d, 56, 12, 1000, device, "cosine")
    g = H.Graph(M=16, Ml=0.25, EfSearch=64, Distance=H.CosineDistance, Rng=5, build_mode=H.BUILD_FLAT, screen=0)
    g.reserve(n, d)
    g.add_device(np.arange(n), X.data_ptr(), n, d)
    del X
    S = Searcher(g, B, 10, d, device)
    for _ in range(2):
        S.run(Q, H.MODE_EXACT, 0)
    g.reset_stats()
    gemm, path = [], []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        S.run(Q, H.MODE_EXACT, 0)
        path.append(g.last_kernel_ms())
        gemm.append(g.get_option("last_gemm_ns") * 1e-6)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    g.device_status()
    unc = g.stats()["exact_uncertified"] / steps
    g.close()
    flops = 2.0 * B * n * d
    gm = float(np.mean(gemm))
    return {"workload": "1M x 1536-d cosine exact search, batch 1024, k=10 (recall 1.0: certified canonical top-k)",
            "queries_per_s": round(B / dt, 1), "ms_per_batch": round(dt * 1e3, 3),
            "exact_path_ms": round(float(np.mean(path)), 3), "uncertified_per_batch": unc,
            "roofline": {"bound": "mfma", "kernel": "k_h1_pp16 (fp16 1-product, v_mfma_f32_16x16x32_f16, fused filter records)",
                         "kernel_ms": round(gm, 4), "flops_per_launch": flops,
                         "achieved": round(flops / (gm * 1e-3) / 1e12, 1), "peak": 2500.0, "unit": "TFLOP/s",
                         "frac": round(flops / (gm * 1e-3) / 1e12 / 2500.0, 4), "traffic": None}}


def config_harder(device, batch=16384, efs=(64, 128, 256, 384, 512), xws=(1, 2, 4), build_expand=4, upper_efc=0,
                  fine_efs=(448, 480, 488, 492, 496), opts=None):
    """Harder structured data (verdict item): the bench generator with latent
    dimension 32 instead of 12, 1M x 768 cosine, on the denser graph that data
    needs (M 32, M0 63, efConstruction 512, same heuristic/slack); recall@10
    against the exact path and QPS / HBM fraction of k_search_beam per ef and
    per layer-0 expansion width (search_expand 1 / 2 / 4: the XW best
    unexpanded entries expanded together, their rows fetched in one round
    trip), and the fastest point reaching recall 0.99 (None when none does)."""
    n, d, M0 = 1_000_000, 768, 63
    X = gen_vectors(n, d, 4321, 32, 1000, device, "cosine")
    Q = gen_vectors(batch, d, 4321 + 7777, 32, 1000, device, "cosine")
    kw = dict(ef_construction=512, heuristic=2, keep_pruned=1, prune_alpha_pct=115, build_expand=build_expand,
              upper_efc=upper_efc, screen=1, batch_ratio_pct=20, time_build=1)
    kw.update(opts or {})  # (tools/harder_probe.py: other graph options)
    g = H.Graph(M=32, Ml=0.25, EfSearch=64, Distance=H.CosineDistance, Rng=5, build_mode=H.BUILD_BATCH, m0=M0, **kw)
    g.reserve(n, d)
    bt, _ = timed(lambda: g.add_device(np.arange(n), X.data_ptr(), n, d))
    bs = g.stats()
    del X
    ngt = 4096
    S = Searcher(g, batch, 10, d, device)
    tk, _, tn = (x.clone() for x in Searcher(g, ngt, 10, d, device).run(Q[:ngt], H.MODE_EXACT, 0))
    points = []
    for xw in xws:
        g.set_option("search_expand", xw)
        # the widest expansion also between ef 384 and 512, where recall crosses 0.99 (finer near it)
        for ef in sorted(set(efs) | (set(fine_efs) if xw == max(xws) else set())):
            kk, _, nn = (x.clone() for x in S.run(Q, H.MODE_BEAM, ef))
            r = recall_at_k(kk[:ngt], nn[:ngt], tk, tn, 10)
            g.reset_stats()
            ms = []
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for _ in range(3):
                S.run(Q, H.MODE_BEAM, ef)
                ms.append(g.last_kernel_ms())
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t1) / 3
            st = g.stats()
            alg = (st["search_f32_evals"] * (4 * d + 4) + st["search_screened"] * 2 * d
                   + st["search_expansions"] * 4 * (M0 + 1)) / 3 + batch * 4 * d
            km = float(np.mean(ms))
            points.append({"search_expand": xw, "ef": ef, "recall_at_10": round(r, 4), "qps": round(batch / dt, 1),
                           "kernel_ms": round(km, 3),
                           "dist_evals_per_query": round(st["search_dist_evals"] / 3 / batch, 1),
                           "expansions_per_query": round(st["search_expansions"] / 3 / batch, 1),
                           "visited_resets_per_query": round(st["visited_resets"] / 3 / batch, 2),
                           "roofline_frac": round(alg / (km * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)})
    g.device_status()
    g.close()
    ok = [p_ for p_ in points if p_["recall_at_10"] >= 0.99]
    per_xw = {str(xw): next((p_ for p_ in points if p_["search_expand"] == xw and p_["recall_at_10"] >= 0.99), None)
              for xw in xws}
    out = {"workload": f"1M x 768-d cosine, latent dimension 32 (harder than the headline's 12), M=32 M0=63 "
                       f"efConstruction=512 build_expand={build_expand} upper_efc={upper_efc} (batches of 20 % of "
                       f"the index), beam k=10, "
                       f"{batch} queries/step",
           "build_inserts_per_s": round(n / bt, 1),
           "build": build_roofline(bs, bt, n, d, M0, "cosine"),
           "operating_points": points,
           "at_recall_0.99_per_search_expand": per_xw,
           "at_recall_0.99": max(ok, key=lambda p_: p_["qps"]) if ok else None}
    return out


def oracle_leg(g, Q, truth, k, ef, metric, seconds, device, nparity=1024):
    """Outside every timed region, on one oracle handle holding the engine's
    exported graph (oracle/: test infrastructure, the checker and the CPU
    baseline only):

    parity -- the north star's criterion (recall@k equal, distances within
      1e-5) on `nparity` of the step's queries, for the beam search (the
      headline) and the reference's Search() semantics (compat): the engine's
      lists against the oracle in ORDER_DEV (the engine's summation tree:
      expected bit-identical) and in ORDER_REF (sequential fp32, the
      reference's arithmetic stand-in), recall against the exact path's truth;
    cpu baseline -- the same graph searched on this host on a bounded sample:
      beam single thread (= BatchSearch's loop, graph.go:1075), the reference's
      compat Search single thread, and beam on every usable CPU (concurrent
      Search, graph_benchmark_test.go:70-89)."""
    import oracle as O  # checker / baseline only
    from oracle.parity import compare_lists

    ex = g.export()
    o = O.Graph(metric=O.COSINE if metric == "cosine" else O.EUCLIDEAN, order=O.ORDER_DEV, M=g.M,
                M0=g.get_option("m0"), Ml=g.Ml, EfSearch=ef)
    o.import_graph(**ex)
    del ex
    threads = host_threads()
    B = min(nparity, Q.shape[0], truth[0].shape[0])
    Qp = Q[:B].contiguous()
    Qh = Qp.cpu().numpy()
    tr = (truth[0][:B].cpu().numpy(), truth[1][:B].cpu().numpy())
    gpu = {}
    for tag, mode in (("beam", H.MODE_BEAM), ("compat", H.MODE_COMPAT)):
        gpu[tag] = tuple(x.clone().cpu().numpy() for x in Searcher(g, B, k, Q.shape[1], device).run(Qp, mode, ef))
    g.device_status()
    par = {"queries": B, "k": k, "ef": ef, "criterion": "recall delta <= 0.002, max |dist diff| <= 1e-5 (north_star)"}
    ok = True
    for tag, mode in (("beam", O.MODE_BEAM), ("compat", O.MODE_COMPAT)):
        o.set_order(O.ORDER_DEV)
        dev = compare_lists(gpu[tag], o.search(Qh, k, mode=mode, ef=ef, threads=threads), k, bitwise=True)
        o.set_order(O.ORDER_REF)
        ref = compare_lists(gpu[tag], o.search(Qh, k, mode=mode, ef=ef, threads=threads), k, truth=tr)
        par[tag] = {"order_dev_identical": dev["identical_lists"], "order_ref_identical": ref["identical_lists"],
                    "recall_gpu": ref["recall_a"], "recall_order_ref": ref["recall_b"],
                    "recall_delta": ref["recall_delta"], "max_abs_dist_diff": ref["max_abs_dist_diff"],
                    "common_pairs": ref["common_pairs"]}
        ok = ok and dev["identical_lists"] == 1.0 and ref["recall_delta"] <= 0.002 and ref["max_abs_dist_diff"] <= 1e-5
    par["pass"] = bool(ok)
    # CPU baseline, ORDER_REF
    out = {}
    nq = len(Qh)
    for name, mode, nt, frac in (("beam", O.MODE_BEAM, 1, 0.4), ("compat", O.MODE_COMPAT, 1, 0.3),
                                 ("beam_mt", O.MODE_BEAM, threads, 0.3)):
        chunk = 32 * nt  # 32 queries per thread per call (thread start-up amortised)
        done, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < seconds * frac:  # cycles through the sample
            o.search(Qh[np.arange(done, done + chunk) % nq], k, mode=mode, ef=ef, threads=nt)
            done += chunk
        out[name] = (done / (time.perf_counter() - t0), done, nt)
    return out, par


def summarize(out):
    """the line's key numbers in one small object (each also in its full object above)"""
    cfg = out.get("configs") or {}
    hd = cfg.get("harder_data") or {}
    h99 = hd.get("at_recall_0.99") or {}
    c4 = cfg.get("configs[4]") or {}
    c2 = cfg.get("configs[2]") or {}
    c0 = cfg.get("configs[0]") or {}
    emu = (out.get("shard") or {}).get("emulated") or {}
    sm = {"qps": out["value"], "recall_at_10": out["recall_at_10"], "search_roofline_frac": out["roofline"]["frac"],
          "build_inserts_per_s": out["build"]["inserts_per_s"], "build_roofline_frac": out["build"]["roofline"]["frac"]}
    if h99:
        sm["harder_at_recall_0.99"] = {k: h99.get(k) for k in ("search_expand", "ef", "recall_at_10", "qps",
                                                                "roofline_frac")}
    if c4:
        sm["configs4_ms_per_batch"] = c4.get("ms_per_batch")
        sm["configs4_gemm_frac"] = (c4.get("roofline") or {}).get("frac")
    if c2:
        sm["configs2_inserts_per_s"] = c2.get("inserts_per_s")
        sm["configs2_build_frac"] = (c2.get("roofline") or {}).get("frac")
    if c0:
        sm["configs0_compat_add_per_s"] = c0.get("gpu_compat_add_inserts_per_s")
        sm["configs0_cpu_compat_add_per_s"] = c0.get("cpu_compat_add_inserts_per_s")
    if emu:
        sm["shard_emulated"] = {k: emu.get(k) for k in ("shards", "per_shard_ef", "merged_recall", "projected_qps",
                                                        "ratio_vs_one_index")}
    return sm


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

    def build(off, rng_seed, nrows=None):
        nonlocal sweep
        nrows = a.nbase if nrows is None else nrows
        X = gen_vectors(nrows, a.dim, a.seed, a.intrinsic, a.clusters, device, a.metric, offset=off)
        g = H.Graph(M=a.M, Ml=0.25, EfSearch=a.ef, Distance=metric, Rng=rng_seed, build_mode=H.BUILD_BATCH,
                    m0=a.M0, ef_construction=a.efc, heuristic=2, keep_pruned=a.keep_pruned, prune_alpha_pct=a.alpha,
                    build_expand=a.build_expand, batch_ratio_pct=a.batch_ratio, upper_efc=a.upper_efc,
                    screen=a.screen, time_build=1)
        g.reserve(nrows, a.dim)
        keys = np.arange(off, off + nrows, dtype=np.int64)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.add_device(keys, X.data_ptr(), nrows, a.dim)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if sweep is None and rank == 0 and nrows == a.nbase:
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

    tmarks = [("start", time.perf_counter())]

    def mark(done):  # wall seconds per leg of this run (the line's leg_seconds)
        tmarks.append((done, time.perf_counter()))

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

    def emulate_shards(nsh, Qs, ek, en, one_index_at99):
        """BASELINE configs[3]'s layout emulated on this one GPU: --total-rows as
        `nsh` node-ID range shards, each built as its own handle exactly as rank r
        of an nsh-rank job builds it (build(lo, seed + r, rows)), every query
        searched on every shard (HIP events per shard launch), the per-shard top-k
        merged by k_merge, recall against the exact top-k of the whole set.  Per
        per-shard ef: merged recall, the slowest shard's search, the merge, and
        the projected nsh-GPU step = slowest shard + merge + the all-gather's
        time at an assumed 100 GB/s per rank over xGMI ((nsh - 1) * B * (12k + 4)
        bytes into each rank); the cheapest ef reaching recall 0.99 against the
        one-index layout's (the N = 1 shard leg: the same rows in one graph)."""
        hs = []
        try:
            for r in range(nsh):
                lo_, hi_ = shard_range(a.total_rows, nsh, r)
                h_, bt_, _ = build(lo_, a.seed + r, hi_ - lo_)
                hs.append((h_, bt_, hi_ - lo_))
            B = Qs.shape[0]
            msg = B * (12 * a.k + 4)
            ag_ms = (nsh - 1) * msg / 100e9 * 1e3
            pts = []
            for ef in ([int(x) for x in a.shard_ef_sweep.split(",") if x] if a.shard_ef_sweep else []):
                lists, kms = [], []
                for h_, _, _ in hs:
                    Sx = Searcher(h_, B, a.k, a.dim, device)
                    lists.append(tuple(x.clone() for x in Sx.run(Qs, H.MODE_BEAM, ef)))
                    ms_ = []
                    for _ in range(3):
                        Sx.run(Qs, H.MODE_BEAM, ef)
                        ms_.append(h_.last_kernel_ms())
                    kms.append(float(np.mean(ms_)))
                    h_.device_status()
                ak = torch.stack([x[0] for x in lists])
                ad = torch.stack([x[1] for x in lists])
                an = torch.stack([x[2] for x in lists])
                mk, md, mn = merge_topk(ak, ad, an, a.k)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    merge_topk(ak, ad, an, a.k)
                e1.record()
                torch.cuda.synchronize()
                mms = e0.elapsed_time(e1) / 5
                r_ = recall_at_k(mk[:ngt], mn[:ngt], ek, en, a.k)
                step_ms = max(kms) + mms + ag_ms
                if pts and pts[-1]["merged_recall_at_10"] >= 0.999:
                    break  # (higher ef only adds time)
                pts.append({"per_shard_ef": ef, "merged_recall_at_10": round(r_, 4),
                            "max_shard_search_ms": round(max(kms), 3), "min_shard_search_ms": round(min(kms), 3),
                            "merge_ms": round(mms, 4), "projected_step_ms": round(step_ms, 3),
                            "projected_qps": round(B / (step_ms * 1e-3), 1)})
            best = next((p_ for p_ in pts if p_["merged_recall_at_10"] >= 0.99), None)
            one = one_index_at99["qps"] if one_index_at99 else None
            return {"shards": nsh, "rows_per_shard": hs[0][2], "queries": B,
                    "build_inserts_per_s": round(sum(x[2] for x in hs) / sum(x[1] for x in hs), 1),
                    "all_gather_est_ms": round(ag_ms, 4),
                    "all_gather_model": f"(shards - 1) x {msg} B into each rank at 100 GB/s (xGMI, not measured here)",
                    "operating_points": pts,
                    "per_shard_ef": best["per_shard_ef"] if best else None,
                    "merged_recall": best["merged_recall_at_10"] if best else None,
                    "projected_qps": best["projected_qps"] if best else None,
                    "one_index_at_recall_0.99": one_index_at99,
                    "ratio_vs_one_index": (round(best["projected_qps"] / one, 3) if best and one else None),
                    "what": (f"{nsh} shards of the same {a.total_rows} rows built and searched one after another on "
                             f"one GPU; the projected rate assumes one shard per GPU searching concurrently")}
        finally:
            for h_, _, _ in hs:
                h_.close()
            torch.cuda.empty_cache()

    g = None
    if not shard_only:
        g, build_s, bstats = build(0, a.seed)
        if a.search_expand != 1:
            g.set_option("search_expand", a.search_expand)
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

    mark("replica_index_and_headline")
    # ---- shard layout: rank r owns rows [r*nbase, (r+1)*nbase) of one dataset --------
    shard_out = None
    shard_g = None
    if shard_only or not a.no_shard_leg:
        lo, hi = shard_range(a.total_rows, world, rank)
        if g is not None and lo == 0 and hi == a.nbase:
            gs, sbuild_s, sbstats = g, build_s, bstats  # rank 0's shard is the replica index
        else:
            gs, sbuild_s, sbstats = build(lo, a.seed + rank, hi - lo)
        shard_g = gs
        Qs = gen_vectors(a.batch, a.dim, qseed, a.intrinsic, a.clusters, device, a.metric)  # same on every rank

        def sstep():
            return sharded_search(engine_local_search(gs, a.k, H.MODE_BEAM, a.ef), Qs, a.k)

        sk, sd, sn = (x.clone() for x in sstep())
        # readiness of the N-rank path, readable without trusting prose: how many
        # ranks took part, that the shards cover the dataset, and that every rank
        # merged the same lists (one all_reduce each of max / min of the checksum)
        csum = list_checksum(sk, sd, sn)
        ready = {"ranks_seen": world, "rows_total": hi - lo, "merged_checksum": csum, "checksums_agree": True}
        if world > 1:
            t_ = torch.tensor([1, hi - lo, csum, -csum], dtype=torch.int64, device=device)
            dist.all_reduce(t_[:2])
            mm = t_[2:].clone()
            dist.all_reduce(mm, op=dist.ReduceOp.MAX)
            ready.update(ranks_seen=int(dist.get_world_size()), ranks_reporting=int(t_[0]), rows_total=int(t_[1]),
                         checksums_agree=bool(int(mm[0]) == -int(mm[1])))
        ek, ed, en = sharded_search(engine_local_search(gs, a.k, H.MODE_EXACT, 0), Qs[:ngt], a.k)
        torch.cuda.synchronize()
        srecall = mean_over_ranks(recall_at_k(sk[:ngt], sn[:ngt], ek, en, a.k))
        s_el, s_kms, s_st = timed_steps(sstep, gs)
        skms = float(np.mean(s_kms))
        # the step's phases (HIP events on torch's stream): local search, the packed
        # all-gather (RCCL), the GPU merge -- 0 at one rank (nothing is exchanged)
        ph = {"search": [], "all_gather": [], "merge": []}
        for _ in range(3):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            ev[0].record()
            lk, ld, ln = engine_local_search(gs, a.k, H.MODE_BEAM, a.ef)(Qs)
            ev[1].record()
            if world > 1:
                gk, gd, gn = gather_topk(lk, ld, ln)
                ev[2].record()
                merge_topk(gk, gd, gn, a.k)
            else:
                ev[2].record()
            ev[3].record()
            torch.cuda.synchronize()
            for name, i in (("search", 0), ("all_gather", 1), ("merge", 2)):
                ph[name].append(ev[i].elapsed_time(ev[i + 1]))
        phases = {f"{k_}_ms": round(float(np.mean(v)), 4) for k_, v in ph.items()}
        # operating points of the shard layout (recall vs the sharded exact top-k, QPS of
        # the whole step: search + exchange + merge, max over ranks), so that one 10M
        # index (N = 1) and 8 shards of 1.25M (N = 8) compare at equal recall
        spoints = []
        for ef in ([int(x) for x in a.shard_ef_sweep.split(",") if x] if a.shard_ef_sweep else []):
            step_ef = lambda: sharded_search(engine_local_search(gs, a.k, H.MODE_BEAM, ef), Qs, a.k)  # noqa: E731
            kk_, _, nn_ = (x.clone() for x in step_ef())
            r_ = mean_over_ranks(recall_at_k(kk_[:ngt], nn_[:ngt], ek, en, a.k))
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for _ in range(3):
                step_ef()
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            tt_ = torch.tensor([(time.perf_counter() - t1) / 3], dtype=torch.float64, device=device)
            if world > 1:
                dist.all_reduce(tt_, op=dist.ReduceOp.MAX)
            spoints.append({"ef": ef, "recall_at_10": round(r_, 4), "qps": round(a.batch / tt_.item(), 1),
                            "ms_per_step": round(tt_.item() * 1e3, 3)})
        gs.device_status()
        sat99 = next((p_ for p_ in spoints if p_["recall_at_10"] >= 0.99), None)
        emu = None
        if world == 1 and a.emulate_shards > 1 and spoints:
            mark("shard_leg")
            emu = emulate_shards(a.emulate_shards, Qs, ek, en, sat99)
        shard_out = {
            "value": round(a.batch * a.steps / s_el, 1), "unit": "queries/s",
            "ms_per_step": round(s_el / a.steps * 1e3, 3), "recall_at_10": round(srecall, 4),
            "n_base_total": a.total_rows, "shards": world, "rows_per_shard": hi - lo,
            "queries_per_step": a.batch, "search_kernel_ms": round(skms, 4),
            "exchange": ("none (one shard)" if world == 1 else
                         f"one all-gather of {a.batch * (12 * a.k + 4)} B per rank ({a.backend}), k_merge on the GPU"),
            "recall_reference": "sharded exact search (per-shard MFMA exact + the same gather + merge)",
            "build_inserts_per_s_per_rank": round((hi - lo) / sbuild_s, 1),
            "phases": phases,
            "readiness": ready,
            "operating_points": spoints,
            "at_recall_0.99": sat99,
            "scaling": "strong (fixed total rows; BASELINE configs[3] at 8 ranks)",
        }
        if emu is not None:
            shard_out["emulated"] = emu
        if shard_only:
            g, build_s, bstats, recall, elapsed, kernel_ms, st = gs, sbuild_s, sbstats, srecall, s_el, s_kms, s_st
            Q, S = Qs, Searcher(gs, a.batch, a.k, a.dim, device)
            tk, tn = ek, en

    def build_traffic(n):
        """HBM bytes of the three insert kernels (k_batch_descend, k_batch_search[_mw],
        k_batch_commit) summed over the build, from separate rocprofv3 --pmc passes of
        this same configuration (tools/profile_round.sh), when one is recorded"""
        try:
            pm = json.load(open(a.pmc_build_json))
            want = dict(n=n, dim=a.dim, efc=a.efc, m0=a.M0, keep_pruned=a.keep_pruned, alpha=a.alpha,
                        screen=a.screen, batch_ratio=a.batch_ratio, build_expand=a.build_expand,
                        upper_efc=a.upper_efc, rev=KERNEL_REV)
            if all(pm.get(k) == v for k, v in want.items()):
                return pm.get("hbm_bytes_total")
        except (OSError, ValueError):
            pass
        return None

    shard = shard_only
    g_rows = (shard_out["rows_per_shard"] if shard_only else a.nbase)
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

    mark("shard_emulation" if (shard_out or {}).get("emulated") else "shard_leg")
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
    # the headline ef at the other layer-0 expansion widths (search_expand)
    xpoints = []
    if world == 1 and a.ef_sweep:
        for xw in (1, 2, 4):
            g.set_option("search_expand", xw)
            kk, _, nn = (x.clone() for x in S.run(Q, H.MODE_BEAM, a.ef))
            r = recall_at_k(kk[:ngt], nn[:ngt], tk, tn, a.k)
            g.reset_stats()
            ms = []
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for _ in range(3):
                S.run(Q, H.MODE_BEAM, a.ef)
                ms.append(g.last_kernel_ms())
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t1) / 3
            ab, e_, x_, _, _ = alg_bytes_of(g.stats(), 3)
            km = float(np.mean(ms))
            xpoints.append({"search_expand": xw, "ef": a.ef, "recall_at_10": round(r, 4), "qps": round(a.batch / dt, 1),
                            "kernel_ms": round(km, 4), "expansions_per_query": round(x_ / a.batch, 1),
                            "roofline_frac": round(ab / (km * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)})
        g.set_option("search_expand", a.search_expand)
    # batch-size points (B in {1, 1024, 10000}): the same graph and ef,
    # queries resident in HBM, wall time per batch over a fixed number of batches
    bpoints = []
    if world == 1 and a.batch_sweep:
        for B in [int(x) for x in a.batch_sweep.split(",") if x]:
            B = min(B, a.batch)
            Sb = Searcher(g, B, a.k, a.dim, device)
            Qb = Q[:B].contiguous()
            reps = max(5, min(500, 200_000 // max(B, 1)))
            Sb.run(Qb, H.MODE_BEAM, a.ef)
            dt, _ = timed(lambda: Sb.run(Qb, H.MODE_BEAM, a.ef), reps=reps)
            kb, _, nb = (x.clone() for x in Sb.run(Qb, H.MODE_BEAM, a.ef))
            r = recall_at_k(kb[:ngt], nb[:ngt], tk[:B], tn[:B], a.k) if B <= ngt else None
            bpoints.append({"batch": B, "ms_per_batch": round(dt * 1e3, 4), "qps": round(B / dt, 1),
                            "batches_timed": reps, "recall_at_10": None if r is None else round(r, 4)})
        g.device_status()
    mark("operating_and_batch_points")
    traffic = None
    if os.path.exists(a.pmc_json):
        try:
            pm = json.load(open(a.pmc_json))
            want = dict(n=a.nbase, dim=a.dim, batch=a.batch, ef=a.ef, efc=a.efc, m0=a.M0, keep_pruned=a.keep_pruned,
                        alpha=a.alpha, screen=a.screen, batch_ratio=a.batch_ratio, rev=KERNEL_REV)
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
            "prune_alpha": a.alpha / 100, "batch_ratio_pct": a.batch_ratio, "build_expand": a.build_expand,
            "upper_efc": a.upper_efc,
            "search_expand": a.search_expand,
            "screen": (("fp16"
                        + " row copy rejects candidates whose f32 distance provably exceeds the list's worst; "
                        "every reported distance is f32, results identical to screen=0") if a.screen else "off"),
            "parallelism": f"{'shard' if shard else 'replica'}{world}",
        },
        "recall_at_10": round(recall, 4),
        "parity": ("measured at N=1 (rank 0, outside the timed region): see the N=1 line" if world > 1 else None),
        "roofline": {
            "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "kernel": "k_search_beam", "kernel_ms": round(kms, 4),
            "alg_bytes_per_launch": int(alg_bytes),
            "dist_evals_per_query": round(E / a.batch, 1), "expansions_per_query": round(Xp / a.batch, 1),
            "screened_per_query": round(Sc / a.batch, 1), "f32_evals_per_query": round(F / a.batch, 1),
            "screen_margin": (g.get_option("screen_err_ppb") * 1e-9) if (g is not None and a.screen) else None,
        },
        "build": build_roofline(bstats, build_s, g_rows, a.dim, a.M0, a.metric, build_traffic(g_rows)),
        "sweep": sweep,
        "cpu_baseline": None,
        "operating_points": points,
        "at_recall_0.99": at99,
        "expand_points": xpoints,
        "batch_points": bpoints,
    }
    if shard_out is not None and not shard_only:
        out["shard"] = shard_out
    if rank == 0 and world == 1 and a.cpu_seconds > 0:
        cb, par = oracle_leg(g, Q[: min(a.batch, 4096)], (tk, tn), a.k, a.ef, a.metric, a.cpu_seconds, device)
        ok_ = par.pop("pass")
        par = dict({"oracle": ("oracle/: C restatement of graph.go/heap.go/distance.go (no Go toolchain) on the "
                               "engine's exported graph; ORDER_DEV = the engine's summation tree, ORDER_REF = "
                               "sequential fp32, pinned by tests/golden/reference_goldens.json")}, **par)
        par["pass"] = ok_
        out["parity"] = par
        mark("oracle_parity_and_cpu_baseline")
        out["cpu_baseline"] = {
            "value": round(cb["beam"][0], 2), "unit": "queries/s", "cores": 1, "kind": "port",
            "sample": f"{cb['beam'][1]} searches cycling over 4096 of the step's queries, same 1M graph, oracle "
                      f"beam search (ORDER_REF sequential fp32), single thread, ~{a.cpu_seconds * 0.4:.0f}s time box",
            "compat_search_qps": round(cb["compat"][0], 2), "compat_sample": cb["compat"][1],
            "beam_mt_qps": round(cb["beam_mt"][0], 2), "beam_mt_threads": cb["beam_mt"][2],
            "beam_mt_sample": cb["beam_mt"][1], "host_cpus": os.cpu_count(), "affinity_cpus": host_threads(),
            "cpu_model": cpu_model(),
            "note": ("compat = the reference's Search() semantics on the same 1M graph; beam_mt = concurrent "
                     "Search on every CPU this process may use (graph_benchmark_test.go:70-89)"),
        }
    if rank == 0 and world == 1 and a.configs:
        for h_ in {id(x): x for x in (g, shard_g) if x is not None}.values():
            h_.close()
        torch.cuda.empty_cache()
        which = set(a.configs.split(","))
        cfg = {}
        if "0" in which:
            cfg["configs[0]"] = config0(device, a.cpu_seconds)
            mark("configs0")
        if "2" in which:
            cfg["configs[2]"] = config2(device, a.build_expand)
            mark("configs2")
        if "4" in which:
            cfg["configs[4]"] = config4(device)
            mark("configs4")
        if "h" in which:
            try:  # an auxiliary leg: a failure here is reported, not fatal to the line
                cfg["harder_data"] = config_harder(device, build_expand=a.harder_build_expand,
                                                   upper_efc=a.harder_upper_efc)
            except Exception as e:  # noqa: BLE001
                cfg["harder_data"] = {"error": f"{type(e).__name__}: {e}"}
            mark("harder_data")
        out["configs"] = cfg
    if rank == 0:
        # the measured parity and a compact summary go last, where a reader of the
        # line's tail (the driver keeps the last few KB) finds them
        out["leg_seconds"] = {n_: round(t_ - tmarks[i][1], 1) for i, (n_, t_) in enumerate(tmarks[1:])}
        par_ = out.pop("parity", None)
        out["summary"] = summarize(out)
        out["parity"] = par_
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
