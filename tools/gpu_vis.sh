# GPU box: visited-set forgetting parity tests + the latent-32 high-ef probe
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/visprobe
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread -m gpu tests/test_gpu_visited.py > gpurun_out/visprobe/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/visprobe/pytest.log; exit 1; }
tail -1 gpurun_out/visprobe/pytest.log
PROBE_LATENT=32 PROBE_EFS=64,128,256,512 timeout -k 10 300 python -u tools/search_probe.py vis_entries=4096 vis_entries=5120 vis_entries=3072 > gpurun_out/visprobe/l32_seed.txt 2>&1 || { echo PROBE_FAIL; tail -20 gpurun_out/visprobe/l32_seed.txt; exit 1; }
cat gpurun_out/visprobe/l32_seed.txt
echo ALL_OK
