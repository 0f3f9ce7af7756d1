#!/bin/bash
# GPU box: SQ counters of k_search_beam on the harder-data graph at ef 64 (R = 1)
# and ef 512 (R = 8), one rocprofv3 --pmc pass per counter group.
# Usage: bash tools/hard_pmc.sh TAG
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P="python3 $R/tools/hard_probe.py 64,512 2"
timeout -k 10 200 $P > $O/plain.log 2>&1 || { echo FAIL_PLAIN; tail -5 $O/plain.log; exit 1; }
cat $O/plain.log
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE -d $O/a -o run --output-format csv -- $P > $O/a.log 2>&1 || { echo FAIL_A; tail -5 $O/a.log; exit 2; }
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES -d $O/b -o run --output-format csv -- $P > $O/b.log 2>&1 || { echo FAIL_B; tail -5 $O/b.log; exit 3; }
echo done > $O/status
