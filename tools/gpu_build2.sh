# GPU box: batched insert -- identical-graph tests, then the bench-index build probe
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/build2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_screen.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_configs.py -k "batch or screen or c3 or repair or config" > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
BUILD_BENCH=1 BUILD_OPTS="time_build=1" timeout -k 10 300 python -u tools/build_probe.py 400 > $O/probe.txt 2>&1 || { echo PROBE_FAIL; tail -20 $O/probe.txt; exit 1; }
timeout -k 10 300 python -u tools/build_probe.py 200 64 >> $O/probe.txt 2>&1 || { echo PROBE2_FAIL; tail -20 $O/probe.txt; exit 1; }
cat $O/probe.txt
echo ALL_OK
