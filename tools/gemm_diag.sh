# GPU box: k_scores_ring timing diagnostics (exact_tile 5 = default, 7 no
# epilogue, 8 + no waits/barriers, 9 + no DMA), rocprofv3 kernel stats each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/gemm_diag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for T in 5 7 8 9; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/t$T -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/exact_probe.py 3 $T 5 > $O/t$T.log 2>&1 || { echo FAIL $T; tail -20 $O/t$T.log; exit 1; }
  grep ms_per_batch $O/t$T.log
done
echo ALL_OK
