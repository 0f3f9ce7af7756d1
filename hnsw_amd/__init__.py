"""hnsw_amd -- MI355X-native engine for the TFMV/hnsw hot path.

Distance sweep -> layer-0 greedy/beam search -> M-neighbour selection on insert,
as hand-written HIP kernels for gfx950 behind a C ABI (include/mhnsw.h,
hnsw_amd/libmhnsw.so).  This package is the host-side mirror of the reference's
Go API (Graph, Node, CosineDistance, ...).  There is no CPU fallback.
"""
from ._lib import (BUILD_BATCH, BUILD_COMPAT, BUILD_FLAT, COSINE, EUCLIDEAN, KEY_INT, KEY_INT32, KEY_INT64, KEY_STRING, KEY_UINT32,
                   KEY_UINT64, MODE_BEAM, MODE_COMPAT, MODE_EXACT, HnswError, LIB_PATH, SIGNATURES, load)
from .graph import (DOG_QUERY_HACK, CosineDistance, DistanceFunc, EuclideanDistance, Graph, LoadSavedGraph, MakeNode,
                    NewGraph, NewGraphWithConfig, Node, RegisterDistanceFunc, SavedGraph, SplitMix64Rand, Vector,
                    distance_func_to_name, max_level, merge_topk_device, random_level, sweep_device)
from .adapters import ExactAdapter, ExactIndex, HNSWAdapter

__all__ = [
    "BUILD_BATCH", "BUILD_COMPAT", "BUILD_FLAT", "ExactIndex", "ExactAdapter", "HNSWAdapter", "KEY_STRING", "COSINE", "EUCLIDEAN", "MODE_BEAM", "MODE_COMPAT", "MODE_EXACT", "HnswError",
    "LIB_PATH", "SIGNATURES", "load", "CosineDistance", "DistanceFunc", "EuclideanDistance", "Graph", "MakeNode",
    "NewGraph", "NewGraphWithConfig", "Node", "RegisterDistanceFunc", "Vector", "distance_func_to_name",
    "merge_topk_device", "KEY_INT", "KEY_INT32", "KEY_INT64", "KEY_UINT32", "KEY_UINT64", "LoadSavedGraph",
    "SavedGraph", "sweep_device", "DOG_QUERY_HACK", "SplitMix64Rand", "max_level", "random_level",
]
