# compat staging guard (large M) + compat tests + a 2-rank gloo rehearsal of the driver's N>1 command
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/gpu_r04l.sh || exit 1
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 \
  bench.py --gpus 2 --steps 3 --warmup 1 --one-gpu --backend gloo --ef-sweep '' --batch-sweep '' --cpu-seconds 0 --configs '' \
  > gpurun_out/r04final_n2.json 2> gpurun_out/r04final_n2.err || { echo N2_FAIL; tail -20 gpurun_out/r04final_n2.err; exit 1; }
tail -c 400 gpurun_out/r04final_n2.json
echo ALL_OK
