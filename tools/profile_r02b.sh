# GPU box: round-2 final profile (bench + kernel trace + FETCH/WRITE PMC passes)
# and the visited-set size probe on the latent-32 set at high ef
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/profile_round.sh r02b || exit 1
mkdir -p gpurun_out/visprobe
PROBE_LATENT=32 PROBE_EFS=128,256,512 timeout -k 10 400 python -u tools/search_probe.py vis_log2=12 vis_log2=13 vis_log2=14 > gpurun_out/visprobe/l32.txt 2>&1 || { echo PROBE_FAIL; tail -20 gpurun_out/visprobe/l32.txt; exit 1; }
cat gpurun_out/visprobe/l32.txt
echo ALL_OK
