# GPU box: exact GEMM timing diagnostics, rocprofv3 kernel stats each.
# Usage: tools/gemm_diag.sh [tiles...]  (default 23 24 25 10: k_h1_pp, no epilogue, no DMA, k_h1_gemm; 10-13 k_h1_gemm: no
# epilogue, + no waits/barriers, + no DMA; 5 7 8 9: the same for k_scores_ring)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/gemm_diag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
TILES=${*:-23 24 25 10}
for T in $TILES; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/t$T$SFX -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/exact_probe.py 3 $T ${REPS:-5} > $O/t$T$SFX.log 2>&1 || { echo FAIL $T; tail -20 $O/t$T$SFX.log; exit 1; }
  grep ms_per_batch $O/t$T$SFX.log
done
echo ALL_OK
