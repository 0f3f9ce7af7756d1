# r04d plus the compat Add cycle accounting (tools/libmhnsw_cprof.so)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
MHNSW_LIB=tools/libmhnsw_cprof.so timeout -k 10 120 python tools/cprof_probe.py 10000 128 8 > gpurun_out/r04e_cprof.txt 2>&1 \
  || { echo CPROF_FAIL; tail -20 gpurun_out/r04e_cprof.txt; exit 1; }
grep -v cprof gpurun_out/r04e_cprof.txt
MHNSW_LIB=tools/libmhnsw_cprof.so timeout -k 10 120 python tools/cprof_probe.py 10000 768 8 > gpurun_out/r04e_cprof768.txt 2>&1 \
  || { echo CPROF_FAIL; tail -20 gpurun_out/r04e_cprof768.txt; exit 1; }
bash tools/gpu_r04d.sh
