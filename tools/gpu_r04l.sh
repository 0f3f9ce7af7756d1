# compat walk with rows kept in registers across remove -> replenish: probe + compat/replace/delete GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 python tools/cprof_probe.py 10000 128 8 && timeout -k 10 120 python tools/cprof_probe.py 10000 768 8
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_replace.py tests/test_gpu_configs.py tests/test_gpu_host.py tests/test_gpu_format.py tests/test_gpu_visited.py \
  > gpurun_out/r04l_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/r04l_tests.log; exit 1; }
tail -2 gpurun_out/r04l_tests.log
echo ALL_OK
