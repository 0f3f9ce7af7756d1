"""Secondary BASELINE configs (not the headline line; results go to profiles/):
  config 3: 1M x 768 Euclidean build throughput (batched insert; compat insert
            throughput on a bounded prefix), plus the resulting recall@10.
  config 5: 1M x 1536 cosine, batch 1024, exact MFMA path: queries/s and
            k_scores TFLOP/s.
  config 4: 10M x 768 cosine in 8 node-ID range shards of 1.25M (the per-GPU
            share at 8 GPUs), emulated on ONE GPU: every shard is built and
            searched with the same queries in turn, the 8 top-k lists are merged
            with k_merge; reports per-shard search time, merge time, recall vs
            the sharded exact path, and the projected 8-GPU throughput.
  4m      : the same 10M vectors as ONE index on one GPU (replica layout).
  compat  : the reference's Search() semantics on the GPU vs the oracle on the
            host, same graph.
  config 1: 10k x 128 U[-1,1) cosine, M=16 Ml=0.25 ef=20 k=10:
            compat build (the reference's Add) and compat Search on the GPU
            vs the oracle on one host core, recall of compat and beam search.
  2b      : the headline graph (bench.py defaults) searched at batch 1, 1024,
            10000 and 65536 (SURVEY 8(d) C2 batch sizes): latency and QPS.
  2u      : SURVEY 8(d) C2 stress set: 1M x 768 U[-1,1) cosine, same build
            parameters, recall@10 and QPS per ef in {32, 64, 128, 256}.
Usage: python tools/bench_configs.py [1] [2b] [2u] [3] [5] [4] [4m] [compat]"""
import json
import os
import sys
import time

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import hnsw_amd as H  # noqa: E402
from bench import Searcher, gen_vectors, recall_at_k  # noqa: E402
from hnsw_amd.shard import merge_topk  # noqa: E402

dev = torch.device("cuda")
which = sys.argv[1:] or ["3", "5", "compat"]


def timed(fn, reps=1):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        r = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps, r


if "3" in which:
    n = 1_000_000
    X = gen_vectors(n, 768, 77, 12, 1000, dev, "euclidean")
    Q = gen_vectors(4096, 768, 78, 12, 1000, dev, "euclidean")
    tk = None
    for efc in (64, 200):  # ef (= efConstruction, graph.go:500) = 64; 200 = quality build
        g = H.Graph(M=16, Ml=0.25, EfSearch=64, Distance=H.EuclideanDistance, Rng=5, build_mode=H.BUILD_BATCH,
                    m0=48, ef_construction=efc, heuristic=2)
        g.reserve(n, 768)
        bt, _ = timed(lambda: g.add_device(np.arange(n), X.data_ptr(), n, 768))
        st = g.stats()
        if tk is None:
            tk, td, tn = (x.clone() for x in Searcher(g, 4096, 10, 768, dev).run(Q, H.MODE_EXACT, 0))
        k_, d_, n_ = Searcher(g, 4096, 10, 768, dev).run(Q, H.MODE_BEAM, 64)
        rec = recall_at_k(k_, n_, tk, tn, 10)
        QB = gen_vectors(65536, 768, 79, 12, 1000, dev, "euclidean")
        SB = Searcher(g, 65536, 10, 768, dev)
        SB.run(QB, H.MODE_BEAM, 64)
        g.reset_stats()
        sdt, _ = timed(lambda: SB.run(QB, H.MODE_BEAM, 64), reps=3)
        sst = g.stats()
        g.close()
        ev = st["build_dist_evals"] / n
        print(json.dumps({"config": "configs[2] 1M x 768 Euclidean insert (batched)", "ef_construction": efc,
                          "inserts_per_s": round(n / bt, 1), "seconds": round(bt, 2),
                          "dist_evals_per_insert": round(ev, 1),
                          "recall_at_10_ef64": round(rec, 4), "M": 16, "M0": 48,
                          "l2_search_qps_ef64_batch65536": round(65536 / sdt, 1),
                          "l2_search_screened_per_query": round(sst["search_screened"] / 3 / 65536, 1),
                          "l2_search_f32_evals_per_query": round(sst["search_f32_evals"] / 3 / 65536, 1)}),
              flush=True)
    # compat (graph.go:437-531 semantics, strictly sequential) on a bounded prefix
    nc = int(os.environ.get("COMPAT_PREFIX", 20000))
    gc = H.Graph(M=16, Ml=0.25, EfSearch=20, Distance=H.EuclideanDistance, Rng=5)
    gc.reserve(nc, 768)
    ct, _ = timed(lambda: gc.add_device(np.arange(nc), X.data_ptr(), nc, 768))
    gc.close()
    print(json.dumps({"config": "configs[2] 1M x 768 Euclidean insert (compat)",
                      "compat_inserts_per_s": round(nc / ct, 1), "compat_prefix": nc,
                      "note": "compat = reference Add() semantics, one wave walks inserts in order"}), flush=True)
    del X

if "5" in which:
    n, d, B = 1_000_000, 1536, 1024
    X = gen_vectors(n, d, 55, 12, 1000, dev, "cosine")
    Q = gen_vectors(B, d, 56, 12, 1000, dev, "cosine")
    g = H.Graph(M=16, Ml=0.25, EfSearch=64, Distance=H.CosineDistance, Rng=5, build_mode=H.BUILD_FLAT)
    g.reserve(n, d)
    g.add_device(np.arange(n), X.data_ptr(), n, d)
    S = Searcher(g, B, 10, d, dev)
    flops = 2.0 * B * n * d
    res = {}
    for prec, name in ((3, "fp16x1_fused"), (2, "fp16x2"), (1, "bf16x3"), (0, "f32")):
        g.set_option("exact_precision", prec)
        S.run(Q, H.MODE_EXACT, 0)
        g.reset_stats()
        dt, out = timed(lambda: S.run(Q, H.MODE_EXACT, 0), reps=5)
        res[name] = [x.clone() for x in out]
        kms = g.last_kernel_ms()
        unc = g.stats()["exact_uncertified"] / 5
        print(json.dumps({"config": "configs[4] 1M x 1536 cosine exact, batch 1024", "scores": name,
                          "queries_per_s": round(B / dt, 1), "ms_per_batch": round(dt * 1e3, 3),
                          "exact_path_ms_events": round(kms, 3),
                          "fp32_equiv_tflops_end_to_end": round(flops / dt / 1e12, 1),
                          "uncertified_per_batch": unc, "mfma_f32_peak_tflops": 157.3,
                          "mfma_bf16_dense_peak_tflops": 2500.0, "recall": 1.0}), flush=True)
    same = all(torch.equal(a_, b_) for other in ("bf16x3", "fp16x2", "fp16x1_fused")
               for a_, b_ in zip(res["f32"], res[other]))
    print(json.dumps({"config": "configs[4] exact: f32 vs bf16x3 vs fp16x2 vs fp16x1_fused results", "identical": same}),
          flush=True)
    g.close()
    del X


if "5t" in which:  # bf16x3 GEMM tile variants (exact_tile option), same workload as config 5
    n, d, B = 1_000_000, 1536, 1024
    X = gen_vectors(n, d, 55, 12, 1000, dev, "cosine")
    Q = gen_vectors(B, d, 56, 12, 1000, dev, "cosine")
    g = H.Graph(M=16, Ml=0.25, EfSearch=64, Distance=H.CosineDistance, Rng=5, build_mode=H.BUILD_FLAT)
    g.reserve(n, d)
    g.add_device(np.arange(n), X.data_ptr(), n, d)
    S = Searcher(g, B, 10, d, dev)
    for prec in (3, 1, 2):
        g.set_option("exact_precision", prec)
        for tile in ((1, 2, 3, 4, 5, 6) if prec == 3 else (1, 2, 3)):
            g.set_option("exact_tile", tile)
            S.run(Q, H.MODE_EXACT, 0)
            dt, _ = timed(lambda: S.run(Q, H.MODE_EXACT, 0), reps=5)
            print(json.dumps({"exact_precision": prec, "exact_tile": tile, "ms_per_batch": round(dt * 1e3, 3)}),
                  flush=True)
    g.close()
    del X


def build_index(n, off, seed, efc, X=None):
    if X is None:
        X = gen_vectors(n, 768, 1234, 12, 1000, dev, "cosine", offset=off)
    g = H.Graph(M=16, Ml=0.25, EfSearch=64, Distance=H.CosineDistance, Rng=seed, build_mode=H.BUILD_BATCH, m0=48,
                ef_construction=efc, heuristic=2, keep_pruned=1)
    g.reserve(n, 768)
    bt, _ = timed(lambda: g.add_device(np.arange(off, off + n), X.data_ptr(), n, 768))
    return g, bt


if "4" in which:
    S_, per, B, NGT = 8, 1_250_000, 16384, 2048
    Q = gen_vectors(B, 768, 1234 + 7777, 12, 1000, dev, "cosine")
    lists, truth, ms, builds = [], [], [], []
    for s_ in range(S_):
        g, bt = build_index(per, s_ * per, 1234 + s_, 400)
        S = Searcher(g, B, 10, 768, dev)
        S.run(Q, H.MODE_BEAM, 64)
        dt, res = timed(lambda: S.run(Q, H.MODE_BEAM, 64), reps=3)
        lists.append([x.clone() for x in res])
        truth.append([x.clone() for x in Searcher(g, NGT, 10, 768, dev).run(Q[:NGT], H.MODE_EXACT, 0)])
        ms.append(dt * 1e3)
        builds.append(bt)
        g.close()
        print(f"shard {s_}: build {bt:.1f}s search {dt * 1e3:.2f} ms", flush=True)

    def stack(ls):
        return (torch.stack([x[0] for x in ls]), torch.stack([x[1] for x in ls]), torch.stack([x[2] for x in ls]))

    ak, ad, an = stack(lists)
    merge_topk(ak, ad, an, 10)
    mt, (mk, md, mn) = timed(lambda: merge_topk(ak, ad, an, 10), reps=5)
    tk, td, tn = merge_topk(*stack(truth), 10)
    rec = recall_at_k(mk[:NGT], mn[:NGT], tk, tn, 10)
    gather_bytes = S_ * B * 10 * 12
    print(json.dumps({"config": "configs[3] 10M x 768 cosine, 8 node-ID range shards of 1.25M, emulated on 1 GPU",
                      "batch": B, "ef": 64, "k": 10, "recall_at_10": round(rec, 4),
                      "shard_search_ms": [round(x, 3) for x in ms], "merge_ms": round(mt * 1e3, 3),
                      "shard_build_s": [round(x, 2) for x in builds],
                      "one_gpu_serial_qps": round(B / ((sum(ms) + mt * 1e3) / 1e3), 1),
                      "projected_8gpu_qps": round(B / ((max(ms) + mt * 1e3) / 1e3), 1),
                      "allgather_bytes_per_gpu": gather_bytes,
                      "note": "projection = slowest shard + merge; the RCCL all-gather of the per-shard top-k "
                              "(B*k*12 B per GPU) is not included"}), flush=True)

if "4m" in which:
    n, B, NGT = 10_000_000, 16384, 2048
    X = gen_vectors(n, 768, 1234, 12, 1000, dev, "cosine")
    Q = gen_vectors(B, 768, 1234 + 7777, 12, 1000, dev, "cosine")
    g, bt = build_index(n, 0, 1234, 200, X)
    del X
    print(f"10M build {bt:.1f}s", flush=True)
    tk, td, tn = (x.clone() for x in Searcher(g, NGT, 10, 768, dev).run(Q[:NGT], H.MODE_EXACT, 0))
    S = Searcher(g, B, 10, 768, dev)
    for ef in (64, 96, 128):
        S.run(Q, H.MODE_BEAM, ef)
        g.reset_stats()
        dt, res = timed(lambda: S.run(Q, H.MODE_BEAM, ef), reps=3)
        st = g.stats()
        E = st["search_dist_evals"] / 3 / B
        rec = recall_at_k(res[0][:NGT], res[2][:NGT], tk, tn, 10)
        print(json.dumps({"config": "10M x 768 cosine, one index on 1 GPU (replica layout)", "ef_construction": 200,
                          "build_s": round(bt, 1), "inserts_per_s": round(n / bt, 1), "ef": ef,
                          "qps": round(B / dt, 1), "recall_at_10": round(rec, 4), "dist_evals_per_query": round(E, 1),
                          "screened_per_query": round(st["search_screened"] / 3 / B, 1),
                          "f32_evals_per_query": round(st["search_f32_evals"] / 3 / B, 1)}), flush=True)
    g.close()

if "compat" in which:
    import oracle as O  # CPU baseline only

    n = 200_000
    X = gen_vectors(n, 768, 1234, 12, 1000, dev, "cosine")
    Q = gen_vectors(4096, 768, 9011, 12, 1000, dev, "cosine")
    g = H.Graph(M=16, Ml=0.25, EfSearch=20, Distance=H.CosineDistance, Rng=3, build_mode=H.BUILD_BATCH, m0=16,
                ef_construction=64)
    g.add_device(np.arange(n), X.data_ptr(), n, 768)
    S = Searcher(g, 4096, 10, 768, dev)
    S.run(Q, H.MODE_COMPAT, 20)
    dt, res = timed(lambda: S.run(Q, H.MODE_COMPAT, 20), reps=3)
    gk = res[0].cpu().numpy()
    o = O.Graph(metric=O.COSINE, order=O.ORDER_DEV, M=16, M0=16, Ml=0.25, EfSearch=20)
    o.import_graph(**g.export())
    qn = Q.cpu().numpy()
    t0 = time.perf_counter()
    ok, od, on = o.search(qn[:512], 10, mode=O.MODE_COMPAT, ef=20)
    ct = time.perf_counter() - t0
    same = bool(np.array_equal(ok, gk[:512]))
    print(json.dumps({"config": "compat Search() semantics, 200k x 768 cosine, M=16 ef=20 k=10",
                      "gpu_queries_per_s": round(4096 / dt, 1), "cpu_oracle_queries_per_s_1thread": round(512 / ct, 1),
                      "identical_results_first_512": same}), flush=True)


if "1" in which:
    import oracle as O  # CPU baseline and ground truth only

    rng = np.random.default_rng(42)  # X ~ U[-1,1), seed 42, then the 1000 queries
    n, d, nq = 10_000, 128, 1000
    Xh = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    Qh = rng.uniform(-1, 1, (nq, d)).astype(np.float32)
    keys = np.arange(n, dtype=np.int64)
    g = H.Graph(M=16, Ml=0.25, EfSearch=20, Distance=H.CosineDistance, Rng=42)  # compat build = reference Add
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g.add_arrays(keys, Xh)
    gbuild = time.perf_counter() - t0
    o = O.Graph(metric=O.COSINE, order=O.ORDER_DEV, M=16, Ml=0.25, EfSearch=20)
    o.import_graph(**g.export())
    ek, _, en = o.search(Qh, 10, mode=O.MODE_EXACT)
    Qd = torch.from_numpy(Qh).to(dev)
    S = Searcher(g, nq, 10, d, dev)
    out = {}
    for name, mode in (("compat", H.MODE_COMPAT), ("beam", H.MODE_BEAM)):
        S.run(Qd, mode, 20)
        dt, res = timed(lambda: S.run(Qd, mode, 20), reps=5)
        k_, n_ = res[0].cpu().numpy(), res[2].cpu().numpy()
        rec = float(np.mean([len(set(k_[b, : n_[b]]) & set(ek[b, : en[b]])) / 10 for b in range(nq)]))
        out[name] = (nq / dt, rec, k_)
    t0 = time.perf_counter()
    ok, _, _ = o.search(Qh, 10, mode=O.MODE_COMPAT, ef=20)
    ct = time.perf_counter() - t0
    # the reference's own build on one core (oracle compat insert, same levels)
    lv = O.Graph(metric=O.COSINE, order=O.ORDER_DEV, M=16, Ml=0.25, EfSearch=20, seed=42).preview_levels(2000)
    oc = O.Graph(metric=O.COSINE, order=O.ORDER_DEV, M=16, Ml=0.25, EfSearch=20, seed=42)
    t0 = time.perf_counter()
    oc.add(keys[:2000], Xh[:2000], lv)
    cbuild = 2000 / (time.perf_counter() - t0)
    print(json.dumps({"config": "configs[0] 10k x 128 U[-1,1) cosine, M=16 Ml=0.25 ef=20 k=10, 1000 queries",
                      "gpu_compat_build_inserts_per_s": round(n / gbuild, 1),
                      "cpu_oracle_compat_build_inserts_per_s_1thread_2k_prefix": round(cbuild, 1),
                      "gpu_compat_search_qps": round(out["compat"][0], 1), "compat_recall_at_10": round(out["compat"][1], 4),
                      "cpu_oracle_compat_search_qps_1thread": round(nq / ct, 1),
                      "gpu_compat_identical_to_oracle": bool(np.array_equal(ok, out["compat"][2])),
                      "gpu_beam_ef20_qps": round(out["beam"][0], 1), "beam_ef20_recall_at_10": round(out["beam"][1], 4),
                      "note": "compat recall is the reference algorithm's own (SURVEY A.3 simulated 0.022); "
                              "beam = standard HNSW search on the same graph"}), flush=True)
    g.close()

if "2b" in which:
    n, d = 1_000_000, 768
    X = gen_vectors(n, d, 1234, 12, 1000, dev, "cosine")
    Q = gen_vectors(65536, d, 1234 + 7777, 12, 1000, dev, "cosine")
    g = H.Graph(M=16, Ml=0.25, EfSearch=64, Distance=H.CosineDistance, Rng=1234, build_mode=H.BUILD_BATCH, m0=40,
                ef_construction=400, heuristic=2, keep_pruned=1, prune_alpha_pct=115)
    g.reserve(n, d)
    g.add_device(np.arange(n), X.data_ptr(), n, d)
    del X
    for B in (1, 1024, 10000, 65536):
        S = Searcher(g, B, 10, d, dev)
        S.run(Q[:B], H.MODE_BEAM, 64)
        reps = 200 if B == 1 else (20 if B <= 10000 else 5)
        dt, _ = timed(lambda: S.run(Q[:B], H.MODE_BEAM, 64), reps=reps)
        print(json.dumps({"config": "configs[1] 1M x 768 cosine ef=64 k=10, batch sweep", "batch": B,
                          "ms_per_batch": round(dt * 1e3, 4), "queries_per_s": round(B / dt, 1)}), flush=True)
    g.close()

if "2u" in which:
    n, d, B, NGT = 1_000_000, 768, 65536, 4096
    gen = torch.Generator(device=dev)
    gen.manual_seed(42)
    X = (torch.rand(n, d, generator=gen, device=dev) * 2 - 1).contiguous()
    Q = (torch.rand(B, d, generator=gen, device=dev) * 2 - 1).contiguous()
    g = H.Graph(M=16, Ml=0.25, EfSearch=64, Distance=H.CosineDistance, Rng=1234, build_mode=H.BUILD_BATCH, m0=40,
                ef_construction=400, heuristic=2, keep_pruned=1, prune_alpha_pct=115)
    g.reserve(n, d)
    bt, _ = timed(lambda: g.add_device(np.arange(n), X.data_ptr(), n, d))
    del X
    tk, td, tn = (x.clone() for x in Searcher(g, NGT, 10, d, dev).run(Q[:NGT], H.MODE_EXACT, 0))
    S = Searcher(g, B, 10, d, dev)
    for ef in (32, 64, 128, 256):
        k_, _, n_ = (x.clone() for x in S.run(Q, H.MODE_BEAM, ef))
        dt, _ = timed(lambda: S.run(Q, H.MODE_BEAM, ef), reps=3)
        print(json.dumps({"config": "configs[1] stress: 1M x 768 U[-1,1) cosine (no neighbour structure)",
                          "build_s": round(bt, 1), "ef": ef, "recall_at_10": round(recall_at_k(k_[:NGT], n_[:NGT], tk, tn, 10), 4),
                          "qps": round(B / dt, 1)}), flush=True)
    g.close()
