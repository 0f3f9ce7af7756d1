"""Diagnostic: the test_compat_build_parity[1500-100-0-16-0.25-20] inputs, each
search mode / exact precision on its own."""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

import hnsw_amd as H  # noqa: E402
import oracle as O  # noqa: E402

n, d, metric, M, ml, ef = 1500, 100, 0, 16, 0.25, 20
rng = np.random.default_rng(n + d)
X = rng.uniform(-1, 1, (n, d)).astype(np.float32)
X[n // 3] = 0.0
Q = rng.uniform(-1, 1, (64, d)).astype(np.float32)
keys = rng.permutation(5 * n)[:n].astype(np.int64) - n
lv = O.Graph(metric=metric, order=O.ORDER_DEV, M=M, Ml=ml, EfSearch=ef, seed=77).preview_levels(n)
g = H.Graph(M=M, Ml=ml, EfSearch=ef, Distance=H.CosineDistance)
g.add_arrays(keys, X, levels=lv)
for mode, efq in ((H.MODE_COMPAT, 20), (H.MODE_BEAM, 64), (H.MODE_EXACT, 0)):
    for prec in ((3, 2, 1, 0) if mode == H.MODE_EXACT else (None,)):
        if prec is not None:
            g.set_option("exact_precision", prec)
        try:
            r = g.search_arrays(Q, 10, mode=mode, ef=efq)
            print("ok", mode, prec, r[2][:8], flush=True)
        except Exception as e:  # noqa: BLE001
            print("FAIL", mode, prec, e, flush=True)
g.set_option("screen", 0)
for efq in (10, 64, 100, 200):
    try:
        g.search_arrays(Q, 10, mode=H.MODE_BEAM, ef=efq)
        print("ok beam screen0", efq, flush=True)
    except Exception as e:  # noqa: BLE001
        print("FAIL beam screen0", efq, e, flush=True)
g.set_option("screen", 1)
for efq in (10, 64, 100, 200):
    try:
        g.search_arrays(Q, 10, mode=H.MODE_BEAM, ef=efq)
        print("ok beam screen1", efq, flush=True)
    except Exception as e:  # noqa: BLE001
        print("FAIL beam screen1", efq, e, flush=True)
