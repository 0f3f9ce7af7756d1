# GPU box: recall / QPS operating points of the headline graph recipe on harder
# structured data (latent dimension 32 and 64 instead of the bench's 12)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/latent
for L in 32 64; do
  timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 --cpu-seconds 0 --no-shard-leg --intrinsic $L \
    --ef-sweep 32,64,96,128,160,192,256,320,384,512 > gpurun_out/latent/L$L.json 2> gpurun_out/latent/L$L.err || { echo FAIL $L; tail -20 gpurun_out/latent/L$L.err; exit 1; }
  echo done $L
done
