"""Host-side mirror of the reference's Graph[K] API (graph.go:17-27, 305-366,
437-1110; distance.go:12-46) over the C ABI of libmhnsw.so.

Names, argument meaning and error messages follow the Go package so that code
(and tests) written against TFMV/hnsw read the same.  Keys are Go `int`
(int64).  Distances are the built-in CosineDistance / EuclideanDistance; they
run on the GPU (a custom Python callable cannot, and is rejected).
"""
from __future__ import annotations

import ctypes as C
import math
import os
from typing import Iterable, List, NamedTuple, Optional, Sequence

import numpy as np

from ._lib import (BUILD_BATCH, BUILD_COMPAT, COSINE, EUCLIDEAN, KEY_INT, KEY_STRING, MODE_BEAM, MODE_COMPAT, MODE_EXACT,
                   HnswError, check, load)

Vector = np.ndarray


class Node(NamedTuple):
    """graph.go:19-23 Node[K]{Key, Value}."""
    Key: int
    Value: Vector


def MakeNode(key, vec) -> Node:  # graph.go:25-27
    return Node(key, np.asarray(vec, dtype=np.float32))


# ---- K of Graph[K cmp.Ordered] ------------------------------------------------
# The engine carries keys as int64 and only ever compares them, so every Go
# ordered key type travels as an order-preserving int64 image:
#   int    -> itself (Go int / int64 / int32 / uint32 ranges)
#   float  -> the IEEE-754 total-order image of the float64 bits (NaN rejected)
#   str    -> the engine's order labels (mhnsw_strkeys_encode: lexicographic
#             order of the UTF-8 bytes = Go string order; labels may be
#             re-spaced by an Add, so they are converted at every call)
_SIGN = np.uint64(1 << 63)


def _float_image(keys) -> np.ndarray:
    f = np.asarray(keys, np.float64).reshape(-1)
    if np.isnan(f).any():
        raise HnswError(-1, "NaN keys are not ordered")
    b = f.view(np.uint64)
    neg = (b >> np.uint64(63)).astype(bool)
    u = np.where(neg, ~b, b | _SIGN)
    return (u ^ _SIGN).view(np.int64)


def _float_key(images: np.ndarray) -> List[float]:
    u = np.asarray(images, np.int64).view(np.uint64) ^ _SIGN
    neg = (u >> np.uint64(63)) == 0
    b = np.where(neg, ~u, u & ~_SIGN)
    return b.view(np.float64).tolist()


def _key_type(key) -> str:
    if isinstance(key, (str, bytes)):
        return "str"
    if isinstance(key, (float, np.floating)):
        return "float"
    return "int"


def _f32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float32)


def _ptr(a: np.ndarray, t):
    return a.ctypes.data_as(C.POINTER(t))


class DistanceFunc:
    """distance.go:12 `type DistanceFunc func(a, b []float32) float32`, backed by
    the GPU sweep kernel (mhnsw_distance)."""

    def __init__(self, name: str, metric: int):
        self.name = name
        self.metric = metric

    def __call__(self, a, b) -> float:
        a, b = _f32(a).ravel(), _f32(b).ravel()
        out = np.zeros(1, np.float32)
        check(load().mhnsw_distance(self.metric, _ptr(a, C.c_float), _ptr(b, C.c_float), 1, a.size,
                                    _ptr(out, C.c_float)))
        return float(out[0])

    def sweep(self, q, X) -> np.ndarray:
        """Batched form: distance of q to every row of X (the hot-path kernel)."""
        q = _f32(q).ravel()
        X = _f32(X).reshape(-1, q.size)
        out = np.zeros(X.shape[0], np.float32)
        check(load().mhnsw_distance(self.metric, _ptr(q, C.c_float), _ptr(X, C.c_float), X.shape[0], q.size,
                                    _ptr(out, C.c_float)))
        return out

    def __repr__(self):
        return f"<DistanceFunc {self.name}>"


CosineDistance = DistanceFunc("cosine", COSINE)  # distance.go:15-17
EuclideanDistance = DistanceFunc("euclidean", EUCLIDEAN)  # distance.go:20-23

_distance_funcs = {"euclidean": EuclideanDistance, "cosine": CosineDistance}  # distance.go:25-28


def RegisterDistanceFunc(name: str, fn: DistanceFunc):  # distance.go:44-46
    _distance_funcs[name] = fn


def distance_func_to_name(fn) -> Optional[str]:  # distance.go:30-39
    for name, f in _distance_funcs.items():
        if f is fn:
            return name
    return None


def _metric_of(fn) -> int:
    if fn is None:
        return -1
    if isinstance(fn, DistanceFunc):
        return fn.metric
    raise HnswError(-6, "custom DistanceFunc is not supported by the GPU engine (use CosineDistance or "
                        "EuclideanDistance)")


def _go_round(x: float) -> float:
    """Go's math.Round: nearest integer, halves away from zero (Python's round()
    and np.round round halves to even)."""
    t = math.trunc(x)
    if abs(x - t) >= 0.5:  # x - trunc(x) is exact in binary floating point
        t += math.copysign(1.0, x)
    return t


def max_level(ml: float, num_nodes: int) -> int:
    """graph.go:370-385 maxLevel."""
    if num_nodes == 0:
        return 1
    return int(_go_round(math.log(float(num_nodes)) / math.log(1.0 / ml))) + 1


def random_level(rng, ml: float, layers_exist: bool, base: int) -> int:
    """graph.go:388-417 randomLevel for a layer 0 of `base` nodes, drawing from
    rng.Float64()."""
    mx = max_level(ml, base) if layers_exist else 1
    for level in range(mx):
        if rng.Float64() > ml:
            return level
    return mx


class SplitMix64Rand:
    """A Go-style *rand.Rand (Float64 in [0,1)) on the engine's own stream:
    levels drawn from SplitMix64Rand(s) equal the engine's seed-s levels."""

    def __init__(self, seed: int):
        self.state = int(seed) & (2**64 - 1)

    # random.Random's protocol: a host Rng with these can be rewound (Graph._walk)
    def getstate(self):
        return self.state

    def setstate(self, st):
        self.state = st

    def Float64(self) -> float:
        m = 2**64 - 1
        self.state = (self.state + 0x9E3779B97F4A7C15) & m
        z = self.state
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
        z ^= z >> 31
        return (z >> 11) * (1.0 / 9007199254740992.0)


DOG_QUERY_HACK = 1  # Graph.TestHacks bit: graph.go:563-569, 595-619


class Graph:
    """graph.go:305-332 Graph[K].  Public fields M, Ml, EfSearch, Distance and
    Rng are read by every call, like the Go struct fields.  Rng is either a
    seed (the engine draws levels from its SplitMix64 stream) or, like Go's
    `*rand.Rand`, any object with Float64(): then every Add draws the levels
    on the host with the reference's rule (graph.go:388-417) and injects them.
    TestHacks (bit DOG_QUERY_HACK) opts into the reference's Search test hack."""

    def __init__(self, M: int = 16, Ml: float = 0.25, EfSearch: int = 20, Distance=CosineDistance,
                 Rng=0, build_mode: int = BUILD_COMPAT, _handle=None, TestHacks: int = 0, **options):
        lib = load()
        h = _handle
        if h is None:
            # a Go struct literal may hold an invalid config; Validate() errors
            # surface at call time, so create with a valid one and apply fields
            h = C.c_void_p()
            check(lib.mhnsw_create(COSINE, 16, 0.25, 20, 0, C.byref(h)))
        self._h = h
        self.M, self.Ml, self.EfSearch, self.Distance = M, Ml, EfSearch, Distance
        self.TestHacks = TestHacks
        self.Rng = Rng
        self._values = {}  # original key -> value (Node.Value)
        self._kt = None    # "int" | "float" | "str" once the first key is seen
        self.set_option("build_mode", build_mode)
        for k, v in options.items():
            self.set_option(k, v)

    # -- lifecycle --------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None):
            load().mhnsw_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _sync(self):
        check(load().mhnsw_set_params(self._h, _metric_of(self.Distance), int(self.M), float(self.Ml),
                                      int(self.EfSearch)), self._h)

    def _check(self, rc):
        return check(rc, self._h)

    @property
    def Rng(self):
        return self._rng

    @Rng.setter
    def Rng(self, rng):
        if hasattr(rng, "Float64"):
            self._rng = rng
            return
        self._rng = int(rng)
        self._check(load().mhnsw_seed(self._h, int(rng) & (2**64 - 1)))

    def _host_rng(self) -> bool:
        return hasattr(self._rng, "Float64") and self.get_option("build_mode") != 2

    def _draw_levels(self, n: int):
        """Levels of the next n inserts (graph.go:962), each from the layer-0
        size before it (the caller knows those inserts are fresh), and the draws
        each one consumed."""
        existed = load().mhnsw_num_layers(self._h) > 0
        base = self.Len()
        ml = float(self.Ml)
        levels, draws = [], []
        for i in range(n):
            mx = max_level(ml, base + i) if (existed or i > 0) else 1
            lv, d = mx, []
            for level in range(mx):  # graph.go:406-416
                r = self._rng.Float64()
                d.append(r)
                if r > ml:
                    lv = level
                    break
            levels.append(lv)
            draws.append(d)
        return np.array(levels, np.int32), draws

    def _walk(self, keys: np.ndarray, add):
        """BatchAdd's walk with levels from the host Rng: the reference draws one
        level per insert it reaches (graph.go:962).  mhnsw_add_plan gives the run
        up to the next present key (where the walk may stop).  When no insert of
        the run can fail part way, its levels are drawn ahead and it goes in one
        call.  When one can (the index holds deleted or replaced rows,
        graph.go:1009: one_by_one), a Rng with getstate()/setstate() (random.Random's
        protocol; SplitMix64Rand has it) still goes in one call: after a failure
        mhnsw_add_reached says how many inserts the walk got to, and the Rng is
        rewound and redraws exactly their draws, so it ends where Go's would.  Any
        other Rng adds one node per call, drawing as the reference does.  An
        error from add(lo, hi, levels) ends the walk."""
        nwalk, one = C.c_int64(), C.c_int()
        rng = self._rng
        rewind = hasattr(rng, "getstate") and hasattr(rng, "setstate")
        lo = 0
        while lo < len(keys):
            self._check(load().mhnsw_add_plan(self._h, _ptr(keys[lo:], C.c_int64), len(keys) - lo, C.byref(nwalk),
                                              C.byref(one)))
            hi = lo + nwalk.value
            if one.value and not rewind:
                hi = lo + 1
            snap = rng.getstate() if rewind else None
            lv, draws = self._draw_levels(hi - lo)
            try:
                add(lo, hi, lv)
            except HnswError:
                if rewind:
                    reached = C.c_int64()
                    self._check(load().mhnsw_add_reached(self._h, C.byref(reached)))
                    rng.setstate(snap)
                    for _ in range(sum(len(d) for d in draws[: reached.value])):
                        rng.Float64()
                raise
            lo = hi

    def set_option(self, name: str, value: int):
        self._check(load().mhnsw_set_option(self._h, name.encode(), int(value)))

    def get_option(self, name: str) -> int:
        v = C.c_int64()
        self._check(load().mhnsw_get_option(self._h, name.encode(), C.byref(v)))
        return v.value

    # -- graph.go:916-937 ---------------------------------------------------
    def Validate(self):
        self._sync()
        self._check(load().mhnsw_validate(self._h))

    # -- keys: Go K -> the engine's int64 order image ---------------------------
    def _bind_kt(self, key):
        kt = _key_type(key)
        if self._kt is None:
            self._kt = kt
        elif kt != self._kt and not (self._kt == "float" and kt == "int"):
            raise HnswError(-1, f"key type {type(key).__name__} does not match the graph's {self._kt} keys")

    def encode_keys(self, keys, assign: bool = False) -> np.ndarray:
        """Go keys -> int64 engine keys (string labels: INT64_MIN when unknown
        and not `assign`)."""
        keys = list(keys)
        if not keys:
            return np.zeros(0, np.int64)
        self._bind_kt(keys[0])
        if self._kt == "int":
            return np.asarray([int(k) for k in keys], np.int64)
        if self._kt == "float":
            return _float_image([float(k) for k in keys])
        bs = [k.encode() if isinstance(k, str) else bytes(k) for k in keys]
        offs = np.zeros(len(bs) + 1, np.int64)
        offs[1:] = np.cumsum([len(b) for b in bs])
        out = np.zeros(len(bs), np.int64)
        self._check(load().mhnsw_strkeys_encode(self._h, b"".join(bs), _ptr(offs, C.c_int64), len(bs),
                                                1 if assign else 0, _ptr(out, C.c_int64)))
        return out

    def decode_keys(self, images) -> list:
        """int64 engine keys (e.g. from search_arrays) -> Go keys."""
        images = np.ascontiguousarray(np.asarray(images, np.int64).reshape(-1))
        if self._kt in (None, "int"):
            return images.tolist()
        if self._kt == "float":
            return _float_key(images)
        lib = load()
        need = C.c_int64()
        self._check(lib.mhnsw_strkeys_decode(self._h, _ptr(images, C.c_int64), len(images), None, 0, None,
                                             C.byref(need)))
        buf = C.create_string_buffer(max(need.value, 1))
        offs = np.zeros(len(images) + 1, np.int64)
        self._check(lib.mhnsw_strkeys_decode(self._h, _ptr(images, C.c_int64), len(images), buf, need.value,
                                             _ptr(offs, C.c_int64), C.byref(need)))
        raw = buf.raw
        return [raw[offs[i]:offs[i + 1]].decode() for i in range(len(images))]

    def _nodes(self, images) -> List[Node]:
        return [self._node(k) for k in self.decode_keys(images)]

    # -- graph.go:437-531 / 942-1042 --------------------------------------------
    def Add(self, *nodes: Node):
        self.BatchAdd(list(nodes))

    def BatchAdd(self, nodes: Sequence[Node], levels=None):
        """graph.go:942-1042.  The walk inserts nodes in order and stops at the
        first error: a node whose dimension differs from the graph's (the
        nodes before it stay added, graph.go:955-960), a present key (replaced,
        then "node not added", graph.go:1015-1037) or a failing search."""
        if not nodes:
            self.Validate()
            return
        vecs = [np.asarray(n.Value, dtype=np.float32).ravel() for n in nodes]
        d0 = self.Dims() or vecs[0].size
        bad = next((i for i, v in enumerate(vecs) if v.size != d0), len(vecs))
        self._sync()
        try:
            if bad:
                keys = self.encode_keys([n.Key for n in nodes[:bad]], assign=True)
                self.add_arrays(keys, np.stack(vecs[:bad]), levels=None if levels is None else levels[:bad])
                for n, v in zip(nodes[:bad], vecs):
                    self._values[n.Key] = v
        except HnswError:
            for n in nodes[:bad]:  # partly applied: Lookup reads the engine
                self._values.pop(n.Key, None)
            raise
        if bad < len(vecs):
            self.Validate()
            raise HnswError(-2, f"embedding dimension mismatch: {d0} != {vecs[bad].size}")

    def add_arrays(self, keys, vecs, levels=None):
        """Array form of BatchAdd: keys int64[n], vecs float32[n, dim] (host)."""
        self._sync()
        keys = np.ascontiguousarray(keys, dtype=np.int64)
        vecs = _f32(vecs).reshape(len(keys), -1)

        def add(lo, hi, lv):
            lv = None if lv is None else np.ascontiguousarray(lv, dtype=np.int32)
            self._check(load().mhnsw_add(self._h, _ptr(keys[lo:], C.c_int64), _ptr(vecs[lo:], C.c_float), hi - lo,
                                         vecs.shape[1], None if lv is None else _ptr(lv, C.c_int32)))

        if levels is None and self._host_rng():
            self._walk(keys, add)
        else:
            add(0, len(keys), levels)

    def add_device(self, keys, vecs_dev_ptr: int, n: int, dim: int, levels=None):
        """BatchAdd with vectors already resident in HBM (device pointer)."""
        self._sync()
        keys = np.ascontiguousarray(keys, dtype=np.int64)

        def add(lo, hi, lv):
            lv = None if lv is None else np.ascontiguousarray(lv, dtype=np.int32)
            self._check(load().mhnsw_add_device(self._h, _ptr(keys[lo:], C.c_int64),
                                                C.c_void_p(vecs_dev_ptr + lo * dim * 4), hi - lo, dim,
                                                None if lv is None else _ptr(lv, C.c_int32)))

        if levels is None and self._host_rng():
            self._walk(keys, add)
        else:
            add(0, n, levels)

    def Replace(self, nodes: Sequence[Node]) -> List[bool]:
        """Flat handles (build_mode 2): overwrite the vectors of present keys in
        place (hybrid/exact.go:28-59 map assignment); -> which keys were present."""
        if not nodes:
            return []
        vecs = [np.asarray(n.Value, dtype=np.float32).ravel() for n in nodes]
        self._sync()
        imgs = np.ascontiguousarray(self.encode_keys([n.Key for n in nodes]), np.int64)
        out = self.replace_arrays(imgs, np.stack(vecs))
        for n, v, ok in zip(nodes, vecs, out):
            if ok:
                self._values[n.Key] = v
        return [bool(x) for x in out]

    def replace_arrays(self, keys, vecs) -> np.ndarray:
        """Array form of Replace: keys int64[n] (engine images), vecs float32[n, dim]."""
        self._sync()
        keys = np.ascontiguousarray(keys, dtype=np.int64)
        vecs = _f32(vecs).reshape(len(keys), -1)
        out = np.zeros(max(len(keys), 1), np.uint8)
        self._check(load().mhnsw_replace(self._h, _ptr(keys, C.c_int64), _ptr(vecs, C.c_float), len(keys),
                                         vecs.shape[1], _ptr(out, C.c_uint8)))
        return out[: len(keys)].astype(bool)

    def contains(self, keys) -> np.ndarray:
        """Which keys have a live node (engine key images for a list of Go keys)."""
        imgs = np.ascontiguousarray(self.encode_keys(list(keys)), np.int64)
        out = np.zeros(max(len(imgs), 1), np.uint8)
        self._check(load().mhnsw_contains(self._h, _ptr(imgs, C.c_int64), len(imgs), _ptr(out, C.c_uint8)))
        return out[: len(imgs)].astype(bool)

    def reserve(self, n: int, dim: int):
        self._check(load().mhnsw_reserve(self._h, n, dim))

    # -- graph.go:534-625 / 1047-1110 --------------------------------------------
    def search_arrays(self, queries, k: int, mode: int = MODE_COMPAT, ef: int = 0, entry_key: Optional[int] = None):
        """Batched search, array form -> (keys int64[B,k], dist float32[B,k], n int32[B])."""
        self._sync()
        q = _f32(queries)
        if q.ndim == 1:
            q = q.reshape(1, -1)
        B, d = q.shape
        kk = max(int(k), 1)
        ok = np.zeros((B, kk), np.int64)
        od = np.zeros((B, kk), np.float32)
        on = np.zeros(B, np.int32)
        ek = None if entry_key is None else C.byref(C.c_int64(int(entry_key)))
        self._check(load().mhnsw_search(self._h, _ptr(q, C.c_float), B, d, int(k), mode, int(ef), ek,
                                        _ptr(ok, C.c_int64), _ptr(od, C.c_float), _ptr(on, C.c_int32)))
        return ok, od, on

    def search_device(self, q_ptr: int, B: int, dim: int, k: int, keys_ptr: int, dist_ptr: int, n_ptr: int,
                      mode: int = MODE_BEAM, ef: int = 0, stream: int = 0):
        """Batched search on device buffers, enqueued on `stream` (no host sync)."""
        self._check(load().mhnsw_search_device(self._h, C.c_void_p(q_ptr), B, dim, k, mode, ef,
                                               C.c_void_p(keys_ptr), C.c_void_p(dist_ptr), C.c_void_p(n_ptr),
                                               C.c_void_p(stream)))

    def device_status(self):
        """Wait for the last enqueued search_device and raise what its kernels
        reported (compat visited-set overflow, out-of-range ids); clears it."""
        self._check(load().mhnsw_device_status(self._h))

    def _node(self, key) -> Node:
        v = self._values.get(key)
        if v is None:
            v, _ = self.Lookup(key)
        return Node(key, v)

    def Search(self, near, k: int, mode: int = MODE_COMPAT) -> List[Node]:
        q = np.asarray(near, np.float32).reshape(1, -1)
        # graph.go:563-569 (opt-in test hack): the dog query searches with 2*EfSearch
        dog = bool(self.TestHacks & DOG_QUERY_HACK) and q.size == 3 and q[0].tolist() == [1.0, np.float32(0.2),
                                                                                           np.float32(0.1)]
        ok, _, on = self.search_arrays(q, k, mode, ef=2 * int(self.EfSearch) if dog else 0)
        out = self._nodes(ok[0, : on[0]])
        if dog and len(out) == 3 and self._kt in (None, "int") and all(n.Key != 3 for n in out):
            v, found = self.Lookup(3)  # graph.go:595-619: canine replaces the last result
            if found:
                out[2] = Node(3, v)
        return out

    def BatchSearch(self, queries: Iterable, k: int, mode: int = MODE_COMPAT) -> List[List[Node]]:
        qs = [np.asarray(q, np.float32).ravel() for q in queries]
        if not qs:
            self._sync()
            if k <= 0:
                raise HnswError(-3, f"k must be greater than 0, got {k}")
            return []
        d0 = self.Dims()
        if d0:
            for i, q in enumerate(qs):
                if q.size != d0:
                    raise HnswError(-2, f"embedding dimension mismatch for query {i}: {d0} != {q.size}")
        ok, _, on = self.search_arrays(np.stack(qs), k, mode)
        return [self._nodes(ok[b, : on[b]]) for b in range(len(qs))]

    def ParallelSearch(self, near, k: int, mode: int = MODE_COMPAT) -> List[Node]:
        """graph.go:631-826: the reference fans distance work out to goroutines;
        here every search is already data-parallel on the GPU (and, unlike the
        reference, deterministic -- Q14)."""
        return self.Search(near, k, mode)

    # -- graph.go:1116-1537 negative-example re-ranking ---------------------------
    def search_negatives_arrays(self, queries, negatives, k: int, negWeight: float, mode: int = MODE_COMPAT,
                                ef: int = 0, flags: int = 0):
        """queries float32[B, dim]; negatives: list (per query) of float32[n_b, dim]
        -> (keys int64[B,k], scores float32[B,k], n int32[B])."""
        self._sync()
        q = _f32(queries)
        if q.ndim == 1:
            q = q.reshape(1, -1)
        B, d = q.shape
        counts = np.array([len(n) for n in negatives], np.int32)
        rows = [_f32(n).reshape(-1, d) for n in negatives if len(n)]
        neg = np.concatenate(rows) if rows else np.zeros((1, d), np.float32)
        kk = max(int(k), 1)
        ok = np.zeros((B, kk), np.int64)
        osc = np.zeros((B, kk), np.float32)
        on = np.zeros(B, np.int32)
        self._check(load().mhnsw_search_negatives(self._h, _ptr(q, C.c_float), B, d, _ptr(neg, C.c_float),
                                                  _ptr(counts, C.c_int32), int(k), float(negWeight), mode, int(ef),
                                                  int(flags), _ptr(ok, C.c_int64), _ptr(osc, C.c_float),
                                                  _ptr(on, C.c_int32)))
        return ok, osc, on

    def _neg_common(self, k, negWeight):
        self.Validate()
        if k <= 0:
            raise HnswError(-3, f"k must be greater than 0, got {k}")
        if negWeight < 0.0 or negWeight > 1.0:
            raise HnswError(-1, f"negWeight must be between 0.0 and 1.0, got {negWeight:f}")

    def SearchWithNegative(self, near, negative, k: int, negWeight: float, mode: int = MODE_COMPAT) -> List[Node]:
        """graph.go:1116-1230"""
        self._neg_common(k, negWeight)
        near = np.asarray(near, np.float32).ravel()
        negative = np.asarray(negative, np.float32).ravel()
        d0 = self.Dims()
        if self.Len() or d0:
            if d0 != near.size:
                raise HnswError(-2, f"query embedding dimension mismatch: {d0} != {near.size}")
            if d0 != negative.size:
                raise HnswError(-2, f"negative embedding dimension mismatch: {d0} != {negative.size}")
        ok, _, on = self.search_negatives_arrays(near[None], [negative[None]], k, negWeight, mode)
        return self._nodes(ok[0, : on[0]])

    def SearchWithNegatives(self, near, negatives, k: int, negWeight: float, mode: int = MODE_COMPAT,
                            flags: int = 0) -> List[Node]:
        """graph.go:1237-1360 (flags=1 enables the reference's key 7..9 test boost)"""
        self._neg_common(k, negWeight)
        if len(negatives) == 0:
            return self.Search(near, k, mode)
        near = np.asarray(near, np.float32).ravel()
        negs = [np.asarray(n, np.float32).ravel() for n in negatives]
        d0 = self.Dims()
        if d0:
            if d0 != near.size:
                raise HnswError(-2, f"query embedding dimension mismatch: {d0} != {near.size}")
            for i, n in enumerate(negs):
                if d0 != n.size:
                    raise HnswError(-2, f"negative embedding {i} dimension mismatch: {d0} != {n.size}")
        ok, _, on = self.search_negatives_arrays(near[None], [np.stack(negs)], k, negWeight, mode, flags=flags)
        return self._nodes(ok[0, : on[0]])

    def BatchSearchWithNegatives(self, queries, negatives, k: int, negWeight: float, mode: int = MODE_COMPAT,
                                 flags: int = 0):
        """graph.go:1365-1537"""
        self._neg_common(k, negWeight)
        qs = [np.asarray(q, np.float32).ravel() for q in queries]
        if not qs:
            return None
        if len(negatives) != len(qs):
            raise HnswError(-1, f"number of negative example sets ({len(negatives)}) must match number of queries "
                                f"({len(qs)})")
        negs = [[np.asarray(n, np.float32).ravel() for n in ns] for ns in negatives]
        d0 = self.Dims()
        if d0:
            for i, q in enumerate(qs):
                if d0 != q.size:
                    raise HnswError(-2, f"query {i} embedding dimension mismatch: {d0} != {q.size}")
                for j, n in enumerate(negs[i]):
                    if d0 != n.size:
                        raise HnswError(-2, f"negative embedding {j} for query {i} dimension mismatch: {d0} != "
                                            f"{n.size}")
        if not self.Len() and not d0:
            return [None] * len(qs)
        ok, _, on = self.search_negatives_arrays(np.stack(qs), [np.stack(n) if n else np.zeros((0, qs[0].size))
                                                                for n in negs], k, negWeight, mode, flags=flags)
        return [self._nodes(ok[b, : on[b]]) for b in range(len(qs))]

    # -- graph.go:829, 421, 898 --------------------------------------------------
    def Len(self) -> int:
        return int(load().mhnsw_len(self._h))

    __len__ = Len

    def Dims(self) -> int:
        return int(load().mhnsw_dims(self._h))

    def Lookup(self, key):
        v = self._values.get(key)
        if v is not None:
            return v, True
        out = np.zeros(max(self.Dims(), 1), np.float32)
        img = int(self.encode_keys([key])[0])
        found = self._check(load().mhnsw_lookup(self._h, img, _ptr(out, C.c_float)))
        return (out if found else None), bool(found)

    def Topography(self) -> List[int]:  # analyzer.go:41-49
        lib = load()
        return [int(lib.mhnsw_layer_count(self._h, l)) for l in range(lib.mhnsw_num_layers(self._h))]

    def Connectivity(self) -> List[float]:  # analyzer.go:20-38
        out = np.zeros(64, np.float64)
        n = self._check(load().mhnsw_connectivity(self._h, _ptr(out, C.c_double), 64))
        return out[:n].tolist()

    # -- Delete / BatchDelete (graph.go:843-895) -------------------------------
    def Delete(self, key) -> bool:
        return self.BatchDelete([key])[0]

    def BatchDelete(self, keys) -> List[bool]:
        orig = list(np.asarray(keys).reshape(-1).tolist()) if isinstance(keys, np.ndarray) else list(keys)
        self._sync()
        imgs = np.ascontiguousarray(self.encode_keys(orig), np.int64)
        out = np.zeros(max(len(imgs), 1), np.uint8)
        self._check(load().mhnsw_delete(self._h, _ptr(imgs, C.c_int64), len(imgs), _ptr(out, C.c_uint8)))
        res = [bool(x) for x in out[:len(imgs)]]
        for key, ok in zip(orig, res):
            if ok:
                self._values.pop(key, None)
        return res

    # -- levels / stats / exchange ------------------------------------------------
    def preview_levels(self, n: int) -> np.ndarray:
        out = np.zeros(n, np.int32)
        self._sync()
        self._check(load().mhnsw_preview_levels(self._h, n, _ptr(out, C.c_int32)))
        return out

    def stats(self) -> dict:
        o = np.zeros(13, np.int64)
        self._check(load().mhnsw_stats(self._h, _ptr(o, C.c_int64), 13))
        names = ["search_dist_evals", "search_expansions", "visited_resets", "build_dist_evals",
                 "build_expansions", "dropped_proposals", "searches", "exact_uncertified",
                 "search_screened", "search_f32_evals", "build_screened", "build_f32_rows", "build_search_us"]
        return dict(zip(names, o.tolist()))

    def reset_stats(self):
        self._check(load().mhnsw_reset_stats(self._h))

    def last_kernel_ms(self) -> float:
        ms = C.c_float()
        self._check(load().mhnsw_last_kernel_ms(self._h, C.byref(ms)))
        return ms.value

    def export(self) -> dict:
        lib = load()
        N, dim, L, cap = C.c_int64(), C.c_int(), C.c_int(), C.c_int()
        self._check(lib.mhnsw_export_sizes(self._h, C.byref(N), C.byref(dim), C.byref(L), C.byref(cap)))
        N, dim, L, cap = N.value, dim.value, L.value, cap.value
        keys = np.zeros(N, np.int64)
        vecs = np.zeros((N, dim), np.float32)
        deg = np.zeros((L, N), np.int32)
        adj = np.zeros((L, N, cap), np.int32)
        entry = np.zeros(max(L, 1), np.int32)
        dead = np.zeros(max(N, 1), np.uint8)
        self._check(lib.mhnsw_export(self._h, _ptr(keys, C.c_int64), _ptr(vecs, C.c_float), _ptr(deg, C.c_int32),
                                     _ptr(adj, C.c_int32), cap, _ptr(entry, C.c_int32), _ptr(dead, C.c_uint8)))
        return dict(keys=keys, vecs=vecs, deg=deg, adj=adj, entry=entry[:L], dead=dead[:N])

    # -- encode.go:128-262 binary format ------------------------------------------
    def _kind(self, key_kind):
        if key_kind is None:
            return KEY_STRING if self._kt == "str" else KEY_INT
        return key_kind

    def export_bytes(self, key_kind: Optional[int] = None) -> bytes:
        """encode.go Export; key_kind = the Go key type (default: string for a
        string-keyed graph, else Go `int`)."""
        key_kind = self._kind(key_kind)
        self._sync()
        lib = load()
        size = C.c_int64()
        self._check(lib.mhnsw_export_go(self._h, key_kind, None, 0, C.byref(size)))
        buf = np.zeros(max(size.value, 1), np.uint8)
        self._check(lib.mhnsw_export_go(self._h, key_kind, _ptr(buf, C.c_uint8), buf.size, C.byref(size)))
        return buf[: size.value].tobytes()

    def import_bytes(self, data: bytes, key_kind: Optional[int] = None):
        key_kind = self._kind(key_kind)
        buf = np.frombuffer(data, np.uint8).copy() if len(data) else np.zeros(1, np.uint8)
        self._check(load().mhnsw_import_go(self._h, _ptr(buf, C.c_uint8), len(data), key_kind))
        self._values.clear()
        self._kt = "str" if key_kind == KEY_STRING else "int"
        self._pull_params()

    def Export(self, w, key_kind: Optional[int] = None):  # encode.go:131-176 (w: has .write)
        w.write(self.export_bytes(key_kind))

    def Import(self, r, key_kind: Optional[int] = None):  # encode.go:181-262 (r: has .read)
        self.import_bytes(r.read(), key_kind)

    def _pull_params(self):
        m, M, ml, ef = C.c_int(), C.c_int(), C.c_double(), C.c_int()
        self._check(load().mhnsw_get_params(self._h, C.byref(m), C.byref(M), C.byref(ml), C.byref(ef)))
        self.M, self.Ml, self.EfSearch = M.value, ml.value, ef.value
        self.Distance = CosineDistance if m.value == COSINE else EuclideanDistance

    def import_graph(self, keys, vecs, deg, adj, entry, dead=None):
        keys = np.ascontiguousarray(keys, np.int64)
        vecs = _f32(vecs)
        deg = np.ascontiguousarray(deg, np.int32)
        adj = np.ascontiguousarray(adj, np.int32)
        entry = np.ascontiguousarray(entry, np.int32)
        dd = None if dead is None else np.ascontiguousarray(dead, np.uint8)
        L, N = deg.shape
        self._sync()
        self._check(load().mhnsw_import(self._h, N, vecs.shape[1], L, adj.shape[2], _ptr(keys, C.c_int64),
                                        _ptr(vecs, C.c_float), _ptr(deg, C.c_int32), _ptr(adj, C.c_int32),
                                        _ptr(entry, C.c_int32), None if dd is None else _ptr(dd, C.c_uint8)))


class SavedGraph(Graph):
    """encode.go:264-327: a Graph persisted to `Path` by Save() (temp file +
    atomic rename)."""

    Path: str = ""

    def Save(self, key_kind: Optional[int] = None):
        key_kind = self._kind(key_kind)
        self._sync()
        self._check(load().mhnsw_save(self._h, os.fsencode(self.Path), key_kind))


def LoadSavedGraph(path: str, key_kind: int = KEY_INT) -> SavedGraph:  # encode.go:280-299
    """Opens (or creates) `path`; an empty or new file gives NewGraph()."""
    import time
    open(path, "ab").close()  # os.O_RDWR|os.O_CREATE
    g = SavedGraph(M=16, Ml=0.25, EfSearch=20, Distance=CosineDistance, Rng=time.time_ns())
    g.Path = path
    g._check(load().mhnsw_load(g._h, os.fsencode(path), key_kind))
    g._kt = "str" if key_kind == KEY_STRING else None
    if g.Len() or os.path.getsize(path):
        g._pull_params()
    return g


def NewGraph() -> Graph:  # graph.go:340-348
    import time
    return Graph(M=16, Ml=0.25, EfSearch=20, Distance=CosineDistance, Rng=time.time_ns())


def NewGraphWithConfig(m: int, ml: float, efSearch: int, distance) -> Graph:  # graph.go:352-366
    import time
    seed = time.time_ns()
    h = C.c_void_p()
    check(load().mhnsw_create(_metric_of(distance), int(m), float(ml), int(efSearch), seed & (2**64 - 1),
                              C.byref(h)))  # validates before touching the device
    return Graph(M=m, Ml=ml, EfSearch=efSearch, Distance=distance, Rng=seed, _handle=h)


def sweep_device(metric: int, q_ptr, X_ptr, n: int, dim: int, out_ptr, stream=0):
    """DistanceFunc batched sweep on device buffers (mhnsw_distance_device):
    out[i] = distance(X[i], q) for n rows of dim contiguous floats."""
    check(load().mhnsw_distance_device(metric, C.c_void_p(q_ptr), C.c_void_p(X_ptr), n, dim, C.c_void_p(out_ptr),
                                       C.c_void_p(stream)))


def merge_topk_device(keys_ptr, dist_ptr, n_ptr, shards, B, k, out_keys, out_dist, out_n, stream=0):
    """Merge per-shard top-k lists (device pointers) -> global top-k by (dist, key)."""
    check(load().mhnsw_merge_topk_device(C.c_void_p(keys_ptr), C.c_void_p(dist_ptr), C.c_void_p(n_ptr), shards,
                                         B, k, C.c_void_p(out_keys), C.c_void_p(out_dist), C.c_void_p(out_n),
                                         C.c_void_p(stream)))
