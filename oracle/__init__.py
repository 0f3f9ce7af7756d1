"""TEST INFRASTRUCTURE ONLY -- ctypes view of the CPU restatement (oracle/oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package, and only as the parity checker / timed CPU baseline.  The product
(hnsw_amd/) never imports it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "liboracle.so")

COSINE, EUCLIDEAN = 0, 1
ORDER_REF, ORDER_DEV = 0, 1
MODE_COMPAT, MODE_BEAM, MODE_EXACT = 0, 1, 2

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = C.CDLL(_SO)
        P = C.POINTER
        f32p, i32p, i64p = P(C.c_float), P(C.c_int32), P(C.c_int64)
        L.og_distance.restype = C.c_float
        L.og_distance.argtypes = [C.c_int, C.c_int, f32p, f32p, C.c_int]
        L.og_dev_norm.restype = C.c_float
        L.og_dev_norm.argtypes = [f32p, C.c_int]
        L.og_heap_run.restype = C.c_int
        L.og_heap_run.argtypes = [P(C.c_int), f32p, i32p, C.c_int, f32p, i32p, i32p, P(C.c_int)]
        L.og_max_level.restype = C.c_int
        L.og_max_level.argtypes = [C.c_double, C.c_int64]
        L.og_rng_next.restype = C.c_double
        L.og_rng_next.argtypes = [P(C.c_uint64)]
        L.og_create.restype = C.c_void_p
        L.og_create.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_double, C.c_int, C.c_uint64]
        L.og_destroy.argtypes = [C.c_void_p]
        L.og_last_error.restype = C.c_char_p
        L.og_last_error.argtypes = [C.c_void_p]
        L.og_set_params.argtypes = [C.c_void_p, C.c_int, C.c_double, C.c_int, C.c_int]
        L.og_set_order.argtypes = [C.c_void_p, C.c_int]
        L.og_set_search_expand.argtypes = [C.c_void_p, C.c_int]
        L.og_validate.argtypes = [C.c_void_p]
        L.og_len.restype = C.c_int64
        L.og_len.argtypes = [C.c_void_p]
        L.og_dims.argtypes = [C.c_void_p]
        L.og_num_layers.argtypes = [C.c_void_p]
        L.og_layer_count.restype = C.c_int64
        L.og_layer_count.argtypes = [C.c_void_p, C.c_int]
        L.og_layer_entry.restype = C.c_int32
        L.og_layer_entry.argtypes = [C.c_void_p, C.c_int]
        L.og_random_level.argtypes = [C.c_void_p]
        L.og_preview_levels.argtypes = [C.c_void_p, C.c_int64, i32p]
        L.og_add.argtypes = [C.c_void_p, i64p, f32p, C.c_int64, C.c_int, i32p]
        L.og_search.argtypes = [C.c_void_p, f32p, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_int,
                                i64p, i64p, f32p, i32p]
        L.og_search_mt.argtypes = [C.c_void_p, f32p, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_int,
                                   i64p, i64p, f32p, i32p, C.c_int]
        L.og_layer_search_compat.argtypes = [C.c_void_p, C.c_int, C.c_int32, C.c_int, C.c_int, f32p,
                                             i32p, f32p]
        L.og_export_sizes.argtypes = [C.c_void_p, i64p, P(C.c_int), P(C.c_int), P(C.c_int)]
        u8p = P(C.c_uint8)
        L.og_export.argtypes = [C.c_void_p, i64p, f32p, i32p, i32p, C.c_int, i32p, u8p]
        L.og_delete.argtypes = [C.c_void_p, i64p, C.c_int64, C.c_int, C.c_int, C.c_int, u8p]
        L.og_import.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.c_int, C.c_int, i64p, f32p, i32p,
                                i32p, i32p, u8p]
        L.og_search_negatives.argtypes = [C.c_void_p, f32p, C.c_int64, C.c_int, f32p, i32p, C.c_int, C.c_float,
                                          C.c_int, C.c_int, C.c_int, i64p, f32p, i32p]
        L.og_stats.argtypes = [C.c_void_p, i64p]
        L.og_reset_stats.argtypes = [C.c_void_p]
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


def f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def distance(metric, order, a, b):
    a, b = f32(a), f32(b)
    return float(lib().og_distance(metric, order, _p(a, C.c_float), _p(b, C.c_float), a.size))


def dev_norm(a):
    a = f32(a)
    return float(lib().og_dev_norm(_p(a, C.c_float), a.size))


def max_level(ml, n):
    return lib().og_max_level(ml, n)


def rng_stream(seed, n):
    s = C.c_uint64(seed)
    return [lib().og_rng_next(C.byref(s)) for _ in range(n)]


def heap_run(ops):
    """ops: list of ('push', d, id) | ('pop',) | ('poplast',) -> (popped ids, heap array)."""
    n = len(ops)
    code = np.array([{"push": 0, "pop": 1, "poplast": 2}[o[0]] for o in ops], dtype=np.int32)
    d = np.array([o[1] if o[0] == "push" else 0 for o in ops], dtype=np.float32)
    ids = np.array([o[2] if o[0] == "push" else 0 for o in ops], dtype=np.int32)
    od = np.zeros(n + 1, np.float32)
    oi = np.zeros(n + 1, np.int32)
    op = np.zeros(n + 1, np.int32)
    npop = C.c_int(0)
    m = lib().og_heap_run(_p(code, C.c_int), _p(d, C.c_float), _p(ids, C.c_int32), n, _p(od, C.c_float),
                          _p(oi, C.c_int32), _p(op, C.c_int32), C.byref(npop))
    return list(op[: npop.value]), list(zip(od[:m].tolist(), oi[:m].tolist()))


class OracleError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(msg)
        self.code = code


class Graph:
    """CPU restatement of hnsw.Graph[int] (graph.go:305-332)."""

    def __init__(self, metric=COSINE, order=ORDER_DEV, M=16, M0=0, Ml=0.25, EfSearch=20, seed=0):
        self._h = lib().og_create(metric, order, M, M0, Ml, EfSearch, seed)
        self.metric = metric

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib is not None:  # module globals may be gone at interpreter exit
            try:
                _lib.og_destroy(h)
            except Exception:
                pass
            self._h = None

    def _check(self, rc):
        if rc != 0:
            raise OracleError(rc, lib().og_last_error(self._h).decode())

    def set_params(self, M, Ml, EfSearch, metric):
        lib().og_set_params(self._h, M, Ml, EfSearch, metric)

    def set_order(self, order):
        """ORDER_REF (sequential fp32, the reference's arithmetic stand-in) or
        ORDER_DEV (the engine's canonical tree) for every later distance."""
        self._check(lib().og_set_order(self._h, order))

    def set_search_expand(self, xw):
        """Beam mode: entries expanded per layer-0 step (1 standard, 2 or 4) --
        the engine's option "search_expand"."""
        self._check(lib().og_set_search_expand(self._h, xw))

    def validate(self):
        self._check(lib().og_validate(self._h))

    def __len__(self):
        return int(lib().og_len(self._h))

    def dims(self):
        return lib().og_dims(self._h)

    def topography(self):
        return [int(lib().og_layer_count(self._h, l)) for l in range(lib().og_num_layers(self._h))]

    def layer_entry(self, l):
        return int(lib().og_layer_entry(self._h, l))

    def random_level(self):
        return lib().og_random_level(self._h)

    def preview_levels(self, n):
        out = np.zeros(n, np.int32)
        lib().og_preview_levels(self._h, n, _p(out, C.c_int32))
        return out

    def add(self, keys, vecs, levels=None):
        keys = np.ascontiguousarray(keys, dtype=np.int64)
        vecs = f32(vecs).reshape(len(keys), -1)
        lv = None if levels is None else np.ascontiguousarray(levels, dtype=np.int32)
        rc = lib().og_add(self._h, _p(keys, C.c_int64), _p(vecs, C.c_float), len(keys), vecs.shape[1],
                          None if lv is None else _p(lv, C.c_int32))
        self._check(rc)

    def search(self, queries, k, mode=MODE_COMPAT, ef=0, entry_key=None, threads=1):
        q = f32(queries)
        if q.ndim == 1:
            q = q.reshape(1, -1)
        B, d = q.shape
        ok = np.zeros((B, max(k, 1)), np.int64)
        od = np.zeros((B, max(k, 1)), np.float32)
        on = np.zeros(B, np.int32)
        ek = None if entry_key is None else C.byref(C.c_int64(entry_key))
        if threads > 1:
            rc = lib().og_search_mt(self._h, _p(q, C.c_float), B, d, k, mode, ef, ek, _p(ok, C.c_int64),
                                    _p(od, C.c_float), _p(on, C.c_int32), threads)
        else:
            rc = lib().og_search(self._h, _p(q, C.c_float), B, d, k, mode, ef, ek, _p(ok, C.c_int64),
                                 _p(od, C.c_float), _p(on, C.c_int32))
        self._check(rc)
        return ok, od, on

    def search_negatives(self, queries, negatives, k, neg_weight, mode=MODE_COMPAT, ef=0, flags=0):
        """graph.go:1116-1537 restated; negatives: list (per query) of [n_b, dim]."""
        q = f32(queries)
        if q.ndim == 1:
            q = q.reshape(1, -1)
        B, d = q.shape
        counts = np.array([len(n) for n in negatives], np.int32)
        rows = [f32(n).reshape(-1, d) for n in negatives if len(n)]
        neg = np.concatenate(rows) if rows else np.zeros((1, d), np.float32)
        kk = max(k, 1)
        ok = np.zeros((B, kk), np.int64)
        osc = np.zeros((B, kk), np.float32)
        on = np.zeros(B, np.int32)
        self._check(lib().og_search_negatives(self._h, _p(q, C.c_float), B, d, _p(neg, C.c_float),
                                              _p(counts, C.c_int32), k, neg_weight, mode, ef, flags,
                                              _p(ok, C.c_int64), _p(osc, C.c_float), _p(on, C.c_int32)))
        return ok, osc, on

    def layer_search_compat(self, layer, entry_id, k, ef, q):
        q = f32(q)
        oi = np.zeros(k + 1, np.int32)
        od = np.zeros(k + 1, np.float32)
        n = lib().og_layer_search_compat(self._h, layer, entry_id, k, ef, _p(q, C.c_float), _p(oi, C.c_int32),
                                         _p(od, C.c_float))
        return oi[:n], od[:n]

    def export(self):
        N, dim, L, cap = C.c_int64(), C.c_int(), C.c_int(), C.c_int()
        lib().og_export_sizes(self._h, C.byref(N), C.byref(dim), C.byref(L), C.byref(cap))
        N, dim, L, cap = N.value, dim.value, L.value, cap.value
        keys = np.zeros(N, np.int64)
        vecs = np.zeros((N, dim), np.float32)
        deg = np.zeros((L, N), np.int32)
        adj = np.zeros((L, N, cap), np.int32)
        entry = np.zeros(max(L, 1), np.int32)
        dead = np.zeros(max(N, 1), np.uint8)
        self._check(lib().og_export(self._h, _p(keys, C.c_int64), _p(vecs, C.c_float), _p(deg, C.c_int32),
                                    _p(adj, C.c_int32), cap, _p(entry, C.c_int32), _p(dead, C.c_uint8)))
        return dict(keys=keys, vecs=vecs, deg=deg, adj=adj, entry=entry[:L], dead=dead[:N])

    def delete(self, keys, mode=0, heuristic=1, keep_pruned=0):
        """Graph.BatchDelete (graph.go:868-895); mode 0 = the reference's
        isolate/replenish, 1 = the engine's batched-graph repair."""
        keys = np.ascontiguousarray(np.atleast_1d(keys), np.int64)
        out = np.zeros(max(len(keys), 1), np.uint8)
        self._check(lib().og_delete(self._h, _p(keys, C.c_int64), len(keys), mode, heuristic, keep_pruned,
                                    _p(out, C.c_uint8)))
        return [bool(x) for x in out[:len(keys)]]

    def import_graph(self, keys, vecs, deg, adj, entry, dead=None):
        keys = np.ascontiguousarray(keys, np.int64)
        vecs = f32(vecs)
        deg = np.ascontiguousarray(deg, np.int32)
        adj = np.ascontiguousarray(adj, np.int32)
        entry = np.ascontiguousarray(entry, np.int32)
        dd = None if dead is None else np.ascontiguousarray(dead, np.uint8)
        L, N = deg.shape
        cap = adj.shape[2]
        self._check(lib().og_import(self._h, N, vecs.shape[1] if vecs.ndim == 2 else 1, L, cap,
                                    _p(keys, C.c_int64), _p(vecs, C.c_float), _p(deg, C.c_int32),
                                    _p(adj, C.c_int32), _p(entry, C.c_int32),
                                    None if dd is None else _p(dd, C.c_uint8)))

    def stats(self):
        o = np.zeros(4, np.int64)
        lib().og_stats(self._h, _p(o, C.c_int64))
        return o.tolist()
