"""TEST INFRASTRUCTURE ONLY -- list-level comparison of two search results.

The north star's parity criterion (BASELINE.json): results match the
reference's Search() on identical inputs -- recall@k equal, distances within
1e-5 fp32.  The reference's arithmetic is restated by the oracle's ORDER_REF
(sequential fp32, vek32's generic path: distance_test.go:12's 0x40a646e1 is
reproduced bitwise); the engine is bit-identical to ORDER_DEV.  This module
measures the ORDER_DEV -> ORDER_REF step on whole result lists:

  identical   fraction of queries whose lists (counts, keys, order) are equal
  recall_*    recall@k of each side against a common exact truth (the
              definition of hybrid/benchmark_test.go:344-361)
  max_abs_dist_diff  largest |d_a - d_b| over (query, key) pairs both lists hold

Used by tests/ and by bench.py's cpu_baseline/parity leg (outside the timed
region); never by the product.
"""
from __future__ import annotations

import numpy as np


def recall(keys, n, tkeys, tn, k):
    tot = 0.0
    for b in range(len(n)):
        t = set(tkeys[b, : tn[b]].tolist())
        tot += len(set(keys[b, : n[b]].tolist()) & t) / max(1, min(k, len(t)))
    return tot / max(1, len(n))


def compare_lists(a, b, k, truth=None, bitwise=False):
    """a, b = (keys[B,k], dist[B,k], n[B]) numpy; truth = (keys, n) or None.
    bitwise: distances must also agree bit for bit for a list to count as
    identical (ORDER_DEV vs the engine); else keys/order/count only."""
    ak, ad, an = (np.asarray(x) for x in a)
    bk, bd, bn = (np.asarray(x) for x in b)
    B = len(an)
    same = 0
    mx = 0.0
    common = 0
    for q in range(B):
        na, nb = int(an[q]), int(bn[q])
        eq = na == nb and np.array_equal(ak[q, :na], bk[q, :nb])
        if eq and bitwise:
            eq = np.array_equal(ad[q, :na].view(np.uint32), bd[q, :nb].view(np.uint32))
        same += bool(eq)
        da = dict(zip(ak[q, :na].tolist(), ad[q, :na].tolist()))
        for key, d in zip(bk[q, :nb].tolist(), bd[q, :nb].tolist()):
            if key in da:
                common += 1
                if np.isfinite(d) and np.isfinite(da[key]):
                    mx = max(mx, abs(float(da[key]) - float(d)))
                elif not (np.isnan(d) and np.isnan(da[key])) and d != da[key]:
                    mx = float("inf")
    out = {"queries": B, "identical_lists": round(same / max(1, B), 6), "common_pairs": common,
           "max_abs_dist_diff": mx}
    if truth is not None:
        tk, tn = (np.asarray(x) for x in truth)
        ra, rb = recall(ak, an, tk, tn, k), recall(bk, bn, tk, tn, k)
        out.update(recall_a=round(ra, 6), recall_b=round(rb, 6), recall_delta=round(abs(ra - rb), 6))
    return out


def same_graph(ea, eb):
    """two exports (keys, deg, adj, entry) describe the same graph: identical
    members, entries and neighbour SETS per row (a row's order is map order)"""
    if not (np.array_equal(ea["keys"], eb["keys"]) and np.array_equal(ea["deg"], eb["deg"])
            and np.array_equal(ea["entry"], eb["entry"])):
        return False
    L, N = ea["deg"].shape
    for l in range(L):
        d = ea["deg"][l]
        rows = np.nonzero(d > 0)[0]
        for i in rows:
            if set(ea["adj"][l, i, : d[i]].tolist()) != set(eb["adj"][l, i, : d[i]].tolist()):
                return False
    return True
