# row prefetch in beam_layer: the full GPU suite and the driver bench command
# the full GPU suite and the driver's bench command (bl_insert DPP shift)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r04j_suite.log 2>&1 \
  || { echo SUITE_FAIL; tail -40 gpurun_out/r04j_suite.log; exit 1; }
tail -2 gpurun_out/r04j_suite.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04j_bench.json 2> gpurun_out/r04j_bench.err \
  || { echo BENCH_FAIL; tail -20 gpurun_out/r04j_bench.err; exit 1; }
echo ALL_OK
