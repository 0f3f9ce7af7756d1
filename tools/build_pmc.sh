#!/bin/bash
# GPU box: where the batched insert's time goes -- SQ counters of k_batch_search on
# the bench index (efC 400), one rocprofv3 --pmc pass per counter group, plus a
# kernel trace of the same build with the selection off (heuristic 0).
# Usage: bash tools/build_pmc.sh TAG
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export BUILD_BENCH=1 BUILD_N=${BUILD_N:-300000}
P="python3 $R/tools/build_probe.py 400"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE -d $O/a -o run --output-format csv -- $P > $O/a.log 2>&1 || { echo FAIL_A; tail -5 $O/a.log; exit 2; }
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES -d $O/b -o run --output-format csv -- $P > $O/b.log 2>&1 || { echo FAIL_B; tail -5 $O/b.log; exit 3; }
BUILD_OPTS="time_build=1,heuristic=0;time_build=1,heuristic=2" timeout -k 10 200 python3 $R/tools/build_probe.py 400 > $O/sel.log 2>&1 || { echo FAIL_SEL; tail -5 $O/sel.log; exit 4; }
grep "^efc" $O/sel.log
echo done > $O/status
