# wide-list batch build at the 4-rows-per-step configs, exact variants / fused fallback, the driver's bench
# command, and a 2-rank shard/replica rehearsal on one GPU (gloo)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_gpu_screen.py::test_batch_build_wide_lists tests/test_gpu_fullsize.py::test_exact_record_variants \
  tests/test_gpu_fullsize.py::test_exact_fused_fallback_segments > gpurun_out/r04d_tests.log 2>&1 \
  || { echo TESTS_FAIL; tail -40 gpurun_out/r04d_tests.log; exit 1; }
tail -2 gpurun_out/r04d_tests.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04d_bench.json 2> gpurun_out/r04d_bench.err \
  || { echo BENCH_FAIL; tail -20 gpurun_out/r04d_bench.err; exit 1; }
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --steps 3 --warmup 1 --one-gpu --backend gloo --ef-sweep '' --batch-sweep '' --cpu-seconds 0 --configs '' \
  > gpurun_out/r04d_n2.json 2> gpurun_out/r04d_n2.err || { echo N2_FAIL; tail -20 gpurun_out/r04d_n2.err; exit 1; }
echo ALL_OK
