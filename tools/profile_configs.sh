#!/bin/bash
# GPU box: secondary configs (3: build, 5: exact) with a kernel-trace profile of each.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-cfg}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/trace5 -o run --output-format csv -- python3 $R/tools/bench_configs.py 5 > $O/cfg5.log 2>&1 || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/trace3 -o run --output-format csv -- python3 $R/tools/bench_configs.py 3 > $O/cfg3.log 2>&1 || exit 2
echo done > $O/status
