# Round-4 GPU call: exact record variants (34 direct, 38 split roles) parity + timing,
# full-size oracle-parity tests, then the driver's bench command.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_gpu_fullsize.py::test_exact_record_variants" \
  > gpurun_out/r04a_rec.log 2>&1 || { echo REC_FAIL; tail -40 gpurun_out/r04a_rec.log; exit 1; }
tail -3 gpurun_out/r04a_rec.log
REPS=20 SFX=_r04a timeout -k 10 700 bash tools/gemm_diag.sh 34 38 31 || exit 1
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_gpu_fullsize.py::test_fullsize_c2_beam tests/test_gpu_fullsize.py::test_fullsize_c3_build \
  tests/test_gpu_fullsize.py::test_fullsize_c5_exact tests/test_gpu_shard.py::test_config3_full_size \
  > gpurun_out/r04a_pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/r04a_pytest.log; exit 1; }
tail -8 gpurun_out/r04a_pytest.log
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04a_bench.json 2> gpurun_out/r04a_bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/r04a_bench.err; exit 1; }
echo ALL_OK
