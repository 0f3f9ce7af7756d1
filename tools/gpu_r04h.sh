# compat Add cycle accounting with the search batches split out
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
MHNSW_LIB=tools/libmhnsw_cprof.so timeout -k 10 120 python tools/cprof_probe.py 10000 128 8 > gpurun_out/r04h_cprof.txt 2>&1 \
  || { echo CPROF_FAIL; tail -20 gpurun_out/r04h_cprof.txt; exit 1; }
grep -v cprof gpurun_out/r04h_cprof.txt
