# compat Add cycle accounting after the global-typed graph loads, LDS layer table, then
# the full GPU suite and the driver's bench command (bl_insert DPP shift)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
MHNSW_LIB=tools/libmhnsw_cprof.so timeout -k 10 120 python tools/cprof_probe.py 10000 128 8 > gpurun_out/r04i_cprof.txt 2>&1 \
  || { echo CPROF_FAIL; tail -20 gpurun_out/r04i_cprof.txt; exit 1; }
grep -v cprof gpurun_out/r04i_cprof.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r04i_suite.log 2>&1 \
  || { echo SUITE_FAIL; tail -40 gpurun_out/r04i_suite.log; exit 1; }
tail -2 gpurun_out/r04i_suite.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04i_bench.json 2> gpurun_out/r04i_bench.err \
  || { echo BENCH_FAIL; tail -20 gpurun_out/r04i_bench.err; exit 1; }
echo ALL_OK
