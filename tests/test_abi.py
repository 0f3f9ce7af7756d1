"""CPU: the C-ABI library loads and exports every symbol include/mhnsw.h
declares; config validation (no device needed) reproduces the reference's
error strings through the ABI."""
import ctypes as C
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "mhnsw.h")).read()
    return sorted(set(re.findall(r"\b(mhnsw_[a-z_]+)\s*\(", src)))


def test_header_matches_binding(H):
    assert _declared() == sorted(H.SIGNATURES)


def test_library_exports_every_symbol(H):
    lib = H.load()
    for name in _declared():
        assert hasattr(lib, name), name


def test_no_cpu_fallback_symbols(H):
    # the product library must not contain or link the oracle
    data = open(H.LIB_PATH, "rb").read()
    assert b"og_search" not in data and b"liboracle" not in data


@pytest.mark.parametrize("M,ml,ef,metric,msg", [
    (0, 0.25, 20, 0, "M must be greater than 0, got 0"),
    (16, 0.0, 20, 0, "Ml must be between 0 and 1 (exclusive), got 0.000000"),
    (16, 1.5, 20, 0, "Ml must be between 0 and 1 (exclusive), got 1.500000"),
    (16, 0.25, 0, 0, "EfSearch must be greater than 0, got 0"),
    (16, 0.25, 20, -1, "Distance function must be set"),
])
def test_create_validation_messages(H, M, ml, ef, metric, msg):
    # NewGraphWithConfig (graph.go:352-366) -> Validate (graph.go:916-937); no device touched
    lib = H.load()
    h = C.c_void_p()
    rc = lib.mhnsw_create(metric, M, ml, ef, 0, C.byref(h))
    assert rc == H._lib.EINVAL
    assert lib.mhnsw_last_error(None).decode() == msg
    assert not h.value


def test_new_graph_with_config_raises(H):
    with pytest.raises(H.HnswError) as e:
        H.NewGraphWithConfig(0, 0.25, 20, H.CosineDistance)
    assert "M must be greater than 0" in str(e.value)
