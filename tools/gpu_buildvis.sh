# GPU box: batched-insert visited-set size probe on the bench index (1M x 768 cosine, efC 400)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/buildvis
BUILD_BENCH=1 BUILD_OPTS="time_build=1;time_build=1,heuristic=0;time_build=1,heuristic=1;time_build=1,keep_pruned=0" timeout -k 10 400 python -u tools/build_probe.py 400 > gpurun_out/buildvis/probe.txt 2>&1 || { echo PROBE_FAIL; tail -20 gpurun_out/buildvis/probe.txt; exit 1; }
cat gpurun_out/buildvis/probe.txt
echo ALL_OK
