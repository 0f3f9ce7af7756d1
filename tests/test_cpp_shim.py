"""GPU: the C++ host shim (include/hnsw_amd/graph.hpp) passes the C++ mirror of
the reference's own tests (tests/cpp/graph_test.cpp)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cpp_build_links_abi():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp")])
    out = subprocess.run(["ldd", os.path.join(ROOT, "tests", "cpp", "graph_test")], capture_output=True, text=True)
    assert "libmhnsw.so" in out.stdout


@pytest.mark.gpu
def test_cpp_shim_reference_tests():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp")])
    r = subprocess.run([os.path.join(ROOT, "tests", "cpp", "graph_test")], capture_output=True, text=True,
                       timeout=300)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASS" in r.stdout
