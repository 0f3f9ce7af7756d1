# compat Add with every walk function inlined (no calls, no scratch): cycle
# accounting, the probe at 128-d / 768-d, and the GPU tests that build compat graphs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
MHNSW_LIB=tools/libmhnsw_cprof.so timeout -k 10 120 python tools/cprof_probe.py 10000 128 8 > gpurun_out/r04g_cprof.txt 2>&1 \
  || { echo CPROF_FAIL; tail -20 gpurun_out/r04g_cprof.txt; exit 1; }
grep -v cprof gpurun_out/r04g_cprof.txt
timeout -k 10 120 python tools/cprof_probe.py 10000 128 8 && timeout -k 10 120 python tools/cprof_probe.py 10000 768 8 \
  && timeout -k 10 120 python tools/cprof_probe.py 10000 128 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_replace.py tests/test_gpu_configs.py tests/test_gpu_host.py tests/test_gpu_format.py tests/test_gpu_visited.py \
  > gpurun_out/r04g_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/r04g_tests.log; exit 1; }
tail -2 gpurun_out/r04g_tests.log
echo ALL_OK
