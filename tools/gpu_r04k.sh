# small-batch multi-wave beam kernel: its parity tests first, then the full suite and the driver bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_latency.py > gpurun_out/r04k_lat.log 2>&1 \
  || { echo LAT_FAIL; tail -40 gpurun_out/r04k_lat.log; exit 1; }
tail -3 gpurun_out/r04k_lat.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r04k_suite.log 2>&1 \
  || { echo SUITE_FAIL; tail -40 gpurun_out/r04k_suite.log; exit 1; }
tail -2 gpurun_out/r04k_suite.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04k_bench.json 2> gpurun_out/r04k_bench.err \
  || { echo BENCH_FAIL; tail -20 gpurun_out/r04k_bench.err; exit 1; }
echo ALL_OK
