"""TEST INFRASTRUCTURE -- pure-Python restatement of the reference's binary
graph format (encode.go:15-262), used to check the engine's C++ codec
(hnsw_amd/csrc/codec.cpp) byte for byte and to feed Go-format files to the
oracle.

  binaryWrite/binaryRead (encode.go:17-104): a Go `int` is a zig-zag varint
  (binary.PutVarint); string and []float32 are a varint length + bytes / LE
  float32s; everything else (float64 Ml, fixed-width keys) is little-endian
  binary.Write.
  Export (encode.go:131-176): version 1, M, Ml, EfSearch, distance name,
  nLayers, then per layer nNodes and per node key, value, nNeighbors,
  neighbour keys.
  Import (encode.go:181-262): neighbour keys resolve within the same layer;
  unresolved keys become nil entries (dropped by to_csr, as the engine does).
"""
import struct

import numpy as np

KEY_INT, KEY_INT64, KEY_INT32, KEY_UINT64, KEY_UINT32, KEY_STRING = 0, 1, 2, 3, 4, 5
_FIXED = {KEY_INT64: "<q", KEY_INT32: "<i", KEY_UINT64: "<Q", KEY_UINT32: "<I"}


class GoError(Exception):
    pass


def put_varint(x: int) -> bytes:
    ux = (x << 1) & 0xFFFFFFFFFFFFFFFF
    if x < 0:
        ux ^= 0xFFFFFFFFFFFFFFFF
    out = bytearray()
    while ux >= 0x80:
        out.append((ux & 0x7F) | 0x80)
        ux >>= 7
    out.append(ux)
    return bytes(out)


def read_varint(buf: bytes, pos: int):
    x, s = 0, 0
    for i in range(10):
        if pos >= len(buf):
            raise GoError("EOF" if i == 0 else "unexpected EOF")
        b = buf[pos]
        pos += 1
        if b < 0x80:
            if i == 9 and b > 1:
                raise GoError("binary: varint overflows a 64-bit integer")
            x |= b << s
            v = x >> 1
            if x & 1:
                v = ~v
            return v, pos
        x |= (b & 0x7F) << s
        s += 7
    raise GoError("binary: varint overflows a 64-bit integer")


def put_key(k, kind: int) -> bytes:
    if kind == KEY_STRING:  # encode.go:78-87: varint length + bytes
        return put_string(k)
    return put_varint(k) if kind == KEY_INT else struct.pack(_FIXED[kind], k)


def read_key(buf, pos, kind):
    if kind == KEY_INT:
        return read_varint(buf, pos)
    if kind == KEY_STRING:  # encode.go:35-45
        n, pos = read_varint(buf, pos)
        if pos + n > len(buf):
            raise GoError("unexpected EOF")
        return buf[pos:pos + n].decode(), pos + n
    fmt = _FIXED[kind]
    n = struct.calcsize(fmt)
    if pos + n > len(buf):
        raise GoError("EOF" if pos >= len(buf) else "unexpected EOF")
    return struct.unpack_from(fmt, buf, pos)[0], pos + n


def put_string(s: str) -> bytes:
    b = s.encode()
    return put_varint(len(b)) + b


def put_floats(v) -> bytes:
    v = np.ascontiguousarray(v, dtype="<f4")
    return put_varint(v.size) + v.tobytes()


def encode(M, Ml, EfSearch, dist, layers, kind=KEY_INT) -> bytes:
    """layers: list (per layer) of lists of (key, values, neighbour keys)."""
    out = [put_varint(1), put_varint(M), struct.pack("<d", Ml), put_varint(EfSearch), put_string(dist),
           put_varint(len(layers))]
    for nodes in layers:
        out.append(put_varint(len(nodes)))
        for key, val, nbs in nodes:
            out += [put_key(key, kind), put_floats(val), put_varint(len(nbs))]
            out += [put_key(k, kind) for k in nbs]
    return b"".join(out)


def encode_export(ex, M, Ml, EfSearch, dist, kind=KEY_INT, keymap=None) -> bytes:
    """An engine/oracle CSR export in the engine's canonical order: live
    members in id order, neighbour keys ascending (`keymap`: engine key ->
    Go key, e.g. string labels -> strings; order-preserving)."""
    km = keymap or (lambda x: x)
    keys, vecs, deg, adj = ex["keys"], ex["vecs"], ex["deg"], ex["adj"]
    dead = ex.get("dead", np.zeros(len(keys), np.uint8))
    layers = []
    for l in range(deg.shape[0]):
        nodes = []
        for i in range(len(keys)):
            if deg[l, i] == -2 or dead[i]:
                continue
            d = max(int(deg[l, i]), 0)
            nodes.append((km(int(keys[i])), vecs[i], [km(k) for k in sorted(int(keys[j]) for j in adj[l, i, :d])]))
        layers.append(nodes)
    return encode(M, Ml, EfSearch, dist, layers, kind)


def decode(buf: bytes, kind=KEY_INT):
    """encode.go:181-262 -> dict(version, M, Ml, EfSearch, dist, layers)."""
    pos = 0
    hdr = []
    for i, what in enumerate(("*int", "*int", "*float64", "*int", "*string")):
        try:
            if what == "*float64":
                if pos + 8 > len(buf):
                    raise GoError("EOF" if pos >= len(buf) else "unexpected EOF")
                v = struct.unpack_from("<d", buf, pos)[0]
                pos += 8
            elif what == "*string":
                n, pos = read_varint(buf, pos)
                if pos + n > len(buf):
                    raise GoError("unexpected EOF")
                v = buf[pos:pos + n].decode()
                pos += n
            else:
                v, pos = read_varint(buf, pos)
        except GoError as e:
            raise GoError(f"reading {what} at index {i}: {e}")
        hdr.append(v)
    version, M, Ml, EfSearch, dist = hdr
    if dist not in ("cosine", "euclidean"):
        raise GoError(f'unknown distance function "{dist}"')
    if version != 1:
        raise GoError(f"incompatible encoding version: {version}")
    nl, pos = read_varint(buf, pos)
    layers = []
    for _ in range(nl):
        nn, pos = read_varint(buf, pos)
        nodes = []
        for j in range(nn):
            key, pos = read_key(buf, pos, kind)
            n, pos = read_varint(buf, pos)
            val = np.frombuffer(buf, dtype="<f4", count=n, offset=pos).astype(np.float32)
            pos += 4 * n
            nnb, pos = read_varint(buf, pos)
            nbs = []
            for _ in range(nnb):
                k, pos = read_key(buf, pos, kind)
                nbs.append(k)
            nodes.append((key, val, nbs))
        layers.append(nodes)
    return dict(version=version, M=M, Ml=Ml, EfSearch=EfSearch, dist=dist, layers=layers)


def to_csr(dec, cap):
    """Decoded file -> import_graph(**) arrays: ids in layer-0 order, neighbours
    resolved within their layer (unresolved dropped), entry = lowest member id,
    a decoded map is never nil (deg >= 0)."""
    layers = dec["layers"]
    L = len(layers)
    keys = np.array([k for k, _, _ in layers[0]], np.int64)
    vecs = np.stack([v for _, v, _ in layers[0]]).astype(np.float32)
    N = len(keys)
    idx = {int(k): i for i, k in enumerate(keys)}
    deg = np.full((L, N), -2, np.int32)
    adj = np.full((L, N, cap), -1, np.int32)
    entry = np.full(L, -1, np.int32)
    for l, nodes in enumerate(layers):
        members = {int(k) for k, _, _ in nodes}
        for key, _, nbs in nodes:
            i = idx[int(key)]
            res = [idx[k] for k in nbs if k in members]
            deg[l, i] = len(res)
            adj[l, i, :len(res)] = res
            entry[l] = i if entry[l] < 0 else min(entry[l], i)
    return dict(keys=keys, vecs=vecs, deg=deg, adj=adj, entry=entry)


def structure(dec):
    """Order-free view for comparisons: per layer {key: sorted neighbour keys}."""
    return [{int(k): sorted(int(x) for x in nbs) for k, _, nbs in nodes} for nodes in dec["layers"]]
