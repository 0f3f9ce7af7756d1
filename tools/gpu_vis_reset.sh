# visited-set reset threshold (3/4 default vs 5/8 vs 1/2) on the harder-data graph at ef 64 / 256 / 512
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for L in hnsw_amd/libmhnsw.so tools/libmhnsw_vis58.so tools/libmhnsw_vis12.so; do
  echo "== $L"
  MHNSW_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 200 python tools/hard_probe.py 64,256,512 3 || exit 1
done
