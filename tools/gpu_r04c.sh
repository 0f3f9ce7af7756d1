# full -m gpu suite; exact GEMM variants (34 / 35, diag 31); batched-insert kernel shapes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 600 --timeout-method thread tests \
  > gpurun_out/r04c_suite.log 2>&1 || { echo SUITE_FAIL; tail -60 gpurun_out/r04c_suite.log; exit 1; }
tail -2 gpurun_out/r04c_suite.log
REPS=20 SFX=_r04c timeout -k 10 400 bash tools/gemm_diag.sh 34 35 || exit 1
MHNSW_LIB=$GRAFT_REPO_ROOT/tools/libmhnsw_diag.so REPS=20 SFX=_r04c timeout -k 10 200 bash tools/gemm_diag.sh 31 || exit 1
for L in hnsw_amd/libmhnsw.so tools/libmhnsw_g4.so tools/libmhnsw_g4w3.so; do
  for V in 12 11; do
    MHNSW_LIB=$GRAFT_REPO_ROOT/$L BUILD_BENCH=1 BUILD_OPTS="vis_log2=$V" timeout -k 10 120 python tools/build_probe.py 400 \
      >> gpurun_out/r04c_build.log 2>&1 || { echo BUILD_FAIL $L; tail -20 gpurun_out/r04c_build.log; exit 1; }
    echo "^ $L vis_log2=$V" >> gpurun_out/r04c_build.log
  done
done
cat gpurun_out/r04c_build.log | grep -v Warn
echo ALL_OK
