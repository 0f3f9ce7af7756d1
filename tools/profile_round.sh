#!/bin/bash
# Runs on the GPU box (via gpurun): rocprofv3 kernel-trace stats of the
# headline phase of the driver's command (its step count, side legs off), and
# separate FETCH_SIZE / WRITE_SIZE PMC passes of the same command and of the
# configs[2] build (the full bench line is tools/gpu_run.sh's bench step).
# Usage: bash tools/profile_round.sh TAG [bench args...]
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
# the driver's step count (--steps 20 --warmup 5): >= 20 launches of the headline kernel, side legs off
PA="--steps 20 --warmup 5 --cpu-seconds 0 --ef-sweep= --batch-sweep= --configs= --no-shard-leg"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py $PA "$@" > $O/trace.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 $R/bench.py $PA "$@" > $O/pmc_fetch.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 $R/bench.py $PA "$@" > $O/pmc_write.log 2>&1 || exit 4
# configs[2] (1M x 768 L2 batched insert, efC 64) alone: its insert kernels' HBM bytes
C2="python3 $R/tools/config2_probe.py 4"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/c2_fetch -o run --output-format csv -- $C2 > $O/c2_fetch.log 2>&1 || exit 5
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/c2_write -o run --output-format csv -- $C2 > $O/c2_write.log 2>&1 || exit 6
echo done > $O/status
