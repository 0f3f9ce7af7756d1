#!/bin/bash
# GPU box: clock / MFMA-busy / wait counters of the exact-path probe for each
# given exact_tile, one rocprofv3 --pmc pass per counter group.
# Usage: bash tools/gemm_pmc.sh TAG tile...
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for T in "$@"; do
  P="python3 $R/tools/exact_probe.py 3 $T 5"
  timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS -d $O/t$T -o run --output-format csv -- $P > $O/t$T.log 2>&1 || { echo FAIL $T; exit 2; }
done
echo done > $O/status
