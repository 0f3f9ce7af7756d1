"""ctypes binding of libmhnsw.so (include/mhnsw.h).

The shared library is built in-tree by __graft_entry__.build() (hipcc, gfx950).
There is no CPU fallback: if the library is missing or cannot be loaded, every
entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# MHNSW_LIB: another build of the same ABI (tools/Makefile.diag's diagnostic library)
LIB_PATH = os.environ.get("MHNSW_LIB") or os.path.join(_HERE, "libmhnsw.so")

COSINE, EUCLIDEAN, NO_DISTANCE = 0, 1, -1
MODE_COMPAT, MODE_BEAM, MODE_EXACT = 0, 1, 2
BUILD_COMPAT, BUILD_BATCH, BUILD_FLAT = 0, 1, 2
KEY_INT, KEY_INT64, KEY_INT32, KEY_UINT64, KEY_UINT32, KEY_STRING = 0, 1, 2, 3, 4, 5

OK, EINVAL, EDIM, EK, ENOMEM, EDEVICE, EUNSUPPORTED, EINTERNAL = 0, -1, -2, -3, -4, -5, -6, -7

#: every symbol include/mhnsw.h declares: name -> (restype, argtypes)
_P = C.POINTER
_f32p, _i32p, _i64p, _vp = _P(C.c_float), _P(C.c_int32), _P(C.c_int64), C.c_void_p
_u8p = _P(C.c_uint8)
SIGNATURES = {
    "mhnsw_create": (C.c_int, [C.c_int, C.c_int, C.c_double, C.c_int, C.c_uint64, _P(_vp)]),
    "mhnsw_destroy": (None, [_vp]),
    "mhnsw_last_error": (C.c_char_p, [_vp]),
    "mhnsw_set_params": (C.c_int, [_vp, C.c_int, C.c_int, C.c_double, C.c_int]),
    "mhnsw_get_params": (C.c_int, [_vp, _P(C.c_int), _P(C.c_int), _P(C.c_double), _P(C.c_int)]),
    "mhnsw_seed": (C.c_int, [_vp, C.c_uint64]),
    "mhnsw_set_option": (C.c_int, [_vp, C.c_char_p, C.c_int64]),
    "mhnsw_get_option": (C.c_int, [_vp, C.c_char_p, _i64p]),
    "mhnsw_validate": (C.c_int, [_vp]),
    "mhnsw_reserve": (C.c_int, [_vp, C.c_int64, C.c_int]),
    "mhnsw_add": (C.c_int, [_vp, _i64p, _f32p, C.c_int64, C.c_int, _i32p]),
    "mhnsw_add_device": (C.c_int, [_vp, _i64p, _vp, C.c_int64, C.c_int, _i32p]),
    "mhnsw_search": (C.c_int, [_vp, _f32p, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_int, _i64p, _i64p, _f32p,
                               _i32p]),
    "mhnsw_search_device": (C.c_int, [_vp, _vp, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_int, _vp, _vp, _vp,
                                      _vp]),
    "mhnsw_device_status": (C.c_int, [_vp]),
    "mhnsw_search_negatives": (C.c_int, [_vp, _f32p, C.c_int64, C.c_int, _f32p, _i32p, C.c_int, C.c_float, C.c_int,
                                         C.c_int, C.c_int, _i64p, _f32p, _i32p]),
    "mhnsw_len": (C.c_int64, [_vp]),
    "mhnsw_dims": (C.c_int, [_vp]),
    "mhnsw_lookup": (C.c_int, [_vp, C.c_int64, _f32p]),
    "mhnsw_contains": (C.c_int, [_vp, _i64p, C.c_int64, _u8p]),
    "mhnsw_add_plan": (C.c_int, [_vp, _i64p, C.c_int64, C.POINTER(C.c_int64), C.POINTER(C.c_int)]),
    "mhnsw_add_reached": (C.c_int, [_vp, C.POINTER(C.c_int64)]),
    "mhnsw_num_layers": (C.c_int, [_vp]),
    "mhnsw_layer_count": (C.c_int64, [_vp, C.c_int]),
    "mhnsw_connectivity": (C.c_int, [_vp, _P(C.c_double), C.c_int]),
    "mhnsw_delete": (C.c_int, [_vp, _i64p, C.c_int64, _u8p]),
    "mhnsw_replace": (C.c_int, [_vp, _i64p, _f32p, C.c_int64, C.c_int, _u8p]),
    "mhnsw_distance": (C.c_int, [C.c_int, _f32p, _f32p, C.c_int64, C.c_int, _f32p]),
    "mhnsw_distance_device": (C.c_int, [C.c_int, _vp, _vp, C.c_int64, C.c_int, _vp, _vp]),
    "mhnsw_export_sizes": (C.c_int, [_vp, _i64p, _P(C.c_int), _P(C.c_int), _P(C.c_int)]),
    "mhnsw_export": (C.c_int, [_vp, _i64p, _f32p, _i32p, _i32p, C.c_int, _i32p, _u8p]),
    "mhnsw_import": (C.c_int, [_vp, C.c_int64, C.c_int, C.c_int, C.c_int, _i64p, _f32p, _i32p, _i32p, _i32p,
                               _u8p]),
    "mhnsw_export_go": (C.c_int, [_vp, C.c_int, _u8p, C.c_int64, _i64p]),
    "mhnsw_strkeys_encode": (C.c_int, [_vp, C.c_char_p, _i64p, C.c_int64, C.c_int, _i64p]),
    "mhnsw_strkeys_decode": (C.c_int, [_vp, _i64p, C.c_int64, _vp, C.c_int64, _i64p, _i64p]),
    "mhnsw_import_go": (C.c_int, [_vp, _u8p, C.c_int64, C.c_int]),
    "mhnsw_save": (C.c_int, [_vp, C.c_char_p, C.c_int]),
    "mhnsw_load": (C.c_int, [_vp, C.c_char_p, C.c_int]),
    "mhnsw_preview_levels": (C.c_int, [_vp, C.c_int64, _i32p]),
    "mhnsw_stats": (C.c_int, [_vp, _i64p, C.c_int]),
    "mhnsw_reset_stats": (C.c_int, [_vp]),
    "mhnsw_last_kernel_ms": (C.c_int, [_vp, _P(C.c_float)]),
    "mhnsw_merge_topk_device": (C.c_int, [_vp, _vp, _vp, C.c_int, C.c_int64, C.c_int, _vp, _vp, _vp, _vp]),
}

_lib = None


class HnswError(RuntimeError):
    """Error returned by the engine; message follows the reference wording."""

    def __init__(self, code: int, message: str):
        super().__init__(message)
        self.code = code


def _share_hip_runtime_with_torch():
    """One HIP runtime per process.  torch links its bundled libamdhip64.so by
    file name, so if libmhnsw.so were loaded first (pulling /opt/rocm's copy,
    same soname) torch would load a second runtime that cannot see the GPU.
    Importing torch first makes our NEEDED libamdhip64.so.7 /
    libhsa-runtime64.so.1 resolve to torch's already-loaded copies."""
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def load() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    _share_hip_runtime_with_torch()
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: run __graft_entry__.build() (hipcc --offload-arch=gfx950)")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int, handle=None):
    if rc < 0:
        msg = load().mhnsw_last_error(handle)
        raise HnswError(rc, msg.decode() if msg else f"error {rc}")
    return rc
