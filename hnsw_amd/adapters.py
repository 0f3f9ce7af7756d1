"""hnsw-extensions/hybrid adapters over the GPU engine.

The reference's hybrid index (hnsw-extensions/hybrid) talks to its
sub-indexes through a small SearchableIndex interface (Add, BatchAdd, Search
-> (keys, distances), Delete, BatchDelete, Len, Close; hybrid/adapter.go).
Here those adapters are thin wrappers over the batched GPU paths:

  ExactIndex    hybrid/exact.go:12-176 -- brute force.  Backed by a flat engine
                handle (build_mode BUILD_FLAT: vector store only, no links) and
                the exact path (MFMA preselection, canonical re-rank,
                certificate), so results are the canonical brute force.  Add
                of an existing key replaces its vector (a map assignment in
                the reference, exact.go:28-38).
  HNSWAdapter   hybrid/adapter.go:11-88 -- a Graph.  Search returns the
                engine's distances (the reference recomputes
                a.distance(query, node.Value), adapter.go:62-64: the same
                canonical value).
  ExactAdapter  hybrid/adapter.go:90-170 -- an ExactIndex.

Ties in distance are returned in insertion order (the reference's map order
is unspecified); NaN distances (zero vectors under cosine) are never returned.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np

from ._lib import BUILD_FLAT, MODE_COMPAT, MODE_EXACT, HnswError
from .graph import CosineDistance, Graph, Node


class ExactIndex:
    """hybrid/exact.go ExactIndex[K] on the GPU exact path."""

    def __init__(self, distance=CosineDistance):
        self.distance = distance
        self._g = Graph(M=16, Ml=0.25, EfSearch=20, Distance=distance, build_mode=BUILD_FLAT)

    def Add(self, key, vector) -> None:  # exact.go:28-38
        self.BatchAdd([key], [vector])

    def BatchAdd(self, keys: Sequence, vectors: Sequence) -> None:  # exact.go:41-59
        if len(keys) != len(vectors):
            raise HnswError(-1, f"number of keys ({len(keys)}) does not match number of vectors ({len(vectors)})")
        if not len(keys):
            return
        latest = {}
        for k, v in zip(keys, vectors):  # later entries of one batch win, like successive map stores
            latest[k] = np.asarray(v, np.float32).ravel()
        ks = list(latest)
        # validate the whole batch first, so a failing batch changes nothing
        d0 = self._g.Dims() or latest[ks[0]].size
        for k in ks:
            if latest[k].size != d0:
                raise HnswError(-2, f"embedding dimension mismatch: {d0} != {latest[k].size}")
        # replacement = map assignment: present keys are overwritten in place
        # (the store does not grow), the others are added -- the add first: the
        # replace of validated rows cannot fail on its arguments
        present = self._g.contains(ks) if self._g.Len() else np.zeros(len(ks), bool)
        new = [Node(k, latest[k]) for k, p in zip(ks, present) if not p]
        if new:
            self._g.BatchAdd(new)
        old = [Node(k, latest[k]) for k, p in zip(ks, present) if p]
        if old:
            self._g.Replace(old)

    def Search(self, query, k: int) -> List[Node]:  # exact.go:62-109
        if self.Len() == 0:
            return []
        return self._g.Search(np.asarray(query, np.float32), k, mode=MODE_EXACT)

    def search_batch(self, queries, k: int) -> Tuple[list, np.ndarray, np.ndarray]:
        """Batched form: -> (keys [B][<=k], distances float32[B, k], n int32[B])."""
        ok, od, on = self._g.search_arrays(np.asarray(queries, np.float32), k, mode=MODE_EXACT)
        return [self._g.decode_keys(ok[b, : on[b]]) for b in range(len(on))], od, on

    def Delete(self, key) -> bool:  # exact.go:112-124
        return self._g.Delete(key)

    def BatchDelete(self, keys) -> List[bool]:  # exact.go:127-143
        return self._g.BatchDelete(keys)

    def Len(self) -> int:  # exact.go:146-151
        return self._g.Len()

    def Close(self) -> None:  # exact.go:154-160
        self._g.close()


class HNSWAdapter:
    """hybrid/adapter.go HNSWAdapter[K]: SearchableIndex over a Graph."""

    def __init__(self, graph: Graph, distance=None, mode: int = MODE_COMPAT):
        self.graph, self.distance, self.mode = graph, distance, mode

    def Add(self, key, vector) -> None:
        self.graph.Add(Node(key, np.asarray(vector, np.float32)))

    def BatchAdd(self, keys: Sequence, vectors: Sequence) -> List[Optional[Exception]]:  # adapter.go:36-50
        if len(keys) != len(vectors):
            return [HnswError(-1, f"number of keys ({len(keys)}) does not match number of vectors "
                                  f"({len(vectors)})")]
        errs: List[Optional[Exception]] = []
        for k, v in zip(keys, vectors):
            try:
                self.Add(k, v)
                errs.append(None)
            except HnswError as e:
                errs.append(e)
        return errs

    def Search(self, query, k: int) -> Tuple[list, List[float]]:  # adapter.go:53-68
        try:
            ok, od, on = self.graph.search_arrays(np.asarray(query, np.float32).reshape(1, -1), k, mode=self.mode)
        except HnswError:
            return None, None
        n = int(on[0])
        return self.graph.decode_keys(ok[0, :n]), od[0, :n].tolist()

    def Delete(self, key) -> bool:
        return self.graph.Delete(key)

    def BatchDelete(self, keys) -> List[bool]:
        return self.graph.BatchDelete(keys)

    def Len(self) -> int:
        return self.graph.Len()

    def Close(self) -> None:  # the reference's graph has nothing to close (adapter.go:84-87)
        pass


class ExactAdapter:
    """hybrid/adapter.go ExactAdapter[K]: SearchableIndex over an ExactIndex."""

    def __init__(self, index: ExactIndex):
        self.index = index

    def Add(self, key, vector) -> None:
        self.index.Add(key, vector)

    def BatchAdd(self, keys: Sequence, vectors: Sequence) -> List[Optional[Exception]]:
        try:
            self.index.BatchAdd(keys, vectors)
            return [None] * len(keys)
        except HnswError as e:
            return [e] * max(len(keys), 1)

    def Search(self, query, k: int) -> Tuple[list, List[float]]:
        if self.index.Len() == 0:
            return [], []
        ks, od, on = self.index.search_batch(np.asarray(query, np.float32).reshape(1, -1), k)
        return ks[0], od[0, : on[0]].tolist()

    def Delete(self, key) -> bool:
        return self.index.Delete(key)

    def BatchDelete(self, keys) -> List[bool]:
        return self.index.BatchDelete(keys)

    def Len(self) -> int:
        return self.index.Len()

    def Close(self) -> None:
        self.index.Close()
