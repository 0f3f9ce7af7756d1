"""Debug helper: replay tests/test_gpu_replace.py::test_delete_then_readd and
print per-call row counts on both sides until they diverge."""
import sys
import numpy as np
sys.path.insert(0, '.')
import hnsw_amd as H
import oracle as O

metric = int(sys.argv[1]) if len(sys.argv) > 1 else 1
rng = np.random.default_rng(77 + metric)
n, d, M = 400, 768, 16
X = rng.uniform(-1, 1, (n, d)).astype(np.float32)
Q = rng.uniform(-1, 1, (24, d)).astype(np.float32)
keys = np.arange(n, dtype=np.int64) * 2 + 1
o = O.Graph(metric=metric, order=O.ORDER_DEV, M=M, Ml=0.25, EfSearch=20, seed=31)
g = H.Graph(M=M, Ml=0.25, EfSearch=20, Distance=H.CosineDistance if metric == 0 else H.EuclideanDistance, Rng=31)
o.add(keys, X)
g.add_arrays(keys, X)
gone = [int(k) for k in rng.choice(keys, 120, replace=False)]
print(o.delete(gone) == g.BatchDelete(gone))
back = list(gone)
rng.shuffle(back)
tries = 0
while back and tries < 40:
    tries += 1
    ks, back = back[:10], back[10:]
    V = rng.uniform(-1, 1, (len(ks), d)).astype(np.float32)
    ex0 = o.export()
    lv = o.preview_levels(len(ks))
    e1 = e2 = None
    try:
        o.add(ks, V)
    except O.OracleError as e:
        e1 = str(e)
    try:
        g.add_arrays(np.array(ks), V)
    except H.HnswError as e:
        e2 = str(e)
    eo, eg = o.export(), g.export()
    print("call", tries, ks, "levels", lv.tolist(), e1, e2, "rows", len(eo["keys"]), len(eg["keys"]))
    if len(eo["keys"]) != len(eg["keys"]):
        new = eo["keys"][len(ex0["keys"]):]
        print(" oracle new rows keys", new.tolist(), "deg", eo["deg"][:, len(ex0["keys"]):].T.tolist())
        gnew = eg["keys"][len(ex0["keys"]):]
        print(" engine new rows keys", gnew.tolist(), "deg", eg["deg"][:, len(ex0["keys"]):].T.tolist())
        print(" topo", o.topography(), g.Topography())
        for k in ks:
            print("  key", k, "oracle rows", [i for i, kk in enumerate(eo["keys"]) if kk == k],
                  "engine rows", [i for i, kk in enumerate(eg["keys"]) if kk == k])
        break
    if e1 is not None:
        in0 = {int(k) for i, k in enumerate(eo["keys"]) if eo["dead"][i] == 0 and eo["deg"][0, i] != -2}
        back += [k for k in ks if k not in in0]
