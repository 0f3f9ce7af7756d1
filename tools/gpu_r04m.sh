# compat rows-in-registers (probe + tests), then the batched-insert schedule probe
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/gpu_r04l.sh || exit 1
BUILD_OPTS="batch_min=1;batch_min=256;batch_min=1024;batch_ratio_pct=10;batch_ratio_pct=20;batch_min=2048" \
  timeout -k 10 400 python tools/schedule_probe.py > gpurun_out/r04m_sched.txt 2>&1 || { echo SCHED_FAIL; tail -20 gpurun_out/r04m_sched.txt; exit 1; }
grep inserts gpurun_out/r04m_sched.txt
