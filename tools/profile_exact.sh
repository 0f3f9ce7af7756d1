#!/bin/bash
# GPU box: kernel trace + PMC passes (one counter group per run) of the exact-path probe.
# Usage: bash tools/profile_exact.sh TAG [probe args]
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P="python3 $R/tools/exact_probe.py $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $P > $O/trace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- $P > $O/fetch.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/tcc -o run --output-format csv -- $P > $O/tcc.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $O/sq -o run --output-format csv -- $P > $O/sq.log 2>&1 || exit 4
echo done > $O/status
