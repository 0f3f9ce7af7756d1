# GPU-box check run: -m gpu tests, a short N=1 bench, a 2-rank shard/replica rehearsal on one GPU (gloo)
# usage: bash tools/gpu_checks.sh [pytest-args...]   (default: the whole -m gpu suite)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 tests/cpp/graph_test > gpurun_out/cpp_test.log 2>&1; echo "cpp_test rc=$?"; tail -5 gpurun_out/cpp_test.log
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread "${@:-tests}" > gpurun_out/pytest1.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest1.log; exit 1; }
tail -3 gpurun_out/pytest1.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-seconds 5 > gpurun_out/bench1.json 2> gpurun_out/bench1.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench1.err; exit 1; }
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --one-gpu --backend gloo --ef-sweep '' --cpu-seconds 0 > gpurun_out/n2_1.json 2> gpurun_out/n2_1.err || { echo N2_FAIL; tail -20 gpurun_out/n2_1.err; exit 1; }
echo ALL_OK
