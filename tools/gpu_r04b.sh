# exact GEMM variants: parity (34, 35, 5), then timing under rocprofv3 (34, 35; 31 from the tools build)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_gpu_fullsize.py::test_exact_record_variants" > gpurun_out/r04b_rec.log 2>&1 || { echo REC_FAIL; tail -40 gpurun_out/r04b_rec.log; exit 1; }
tail -3 gpurun_out/r04b_rec.log
REPS=20 SFX=_r04b timeout -k 10 500 bash tools/gemm_diag.sh 34 35 || exit 1
MHNSW_LIB=$GRAFT_REPO_ROOT/tools/libmhnsw_diag.so REPS=20 SFX=_r04b timeout -k 10 300 bash tools/gemm_diag.sh 31 || exit 1
echo ALL_OK
