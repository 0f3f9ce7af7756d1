# round-4 final binary: smoke, the full GPU suite, the driver's bench command
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04final_smoke.log 2>&1 \
  || { echo SMOKE_FAIL; tail -20 gpurun_out/r04final_smoke.log; exit 1; }
tail -1 gpurun_out/r04final_smoke.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r04final_suite.log 2>&1 \
  || { echo SUITE_FAIL; tail -40 gpurun_out/r04final_suite.log; exit 1; }
tail -2 gpurun_out/r04final_suite.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04final_bench.json 2> gpurun_out/r04final_bench.err \
  || { echo BENCH_FAIL; tail -20 gpurun_out/r04final_bench.err; exit 1; }
echo ALL_OK
