# GPU box: screened neighbour selection -- identical-graph tests, build throughput
# (bench index, configs[2]) and a stronger graph on the latent-32 set
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/build
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_screen.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -k "batch or screen or c3 or repair" > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 --cpu-seconds 0 --no-shard-leg --ef-sweep '' > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
python -c "import json; b=json.load(open('$O/bench.json')); print(b['value'], b['recall_at_10'], b['build'])"
timeout -k 10 400 python -u tools/bench_configs.py 3 > $O/cfg3.jsonl 2> $O/cfg3.err || { echo CFG3_FAIL; tail -20 $O/cfg3.err; exit 1; }
cat $O/cfg3.jsonl
timeout -k 10 500 python -u bench.py --steps 5 --warmup 1 --cpu-seconds 0 --no-shard-leg --intrinsic 32 --M 32 --M0 63 --efc 512 \
    --ef-sweep 64,96,128,192,256,384,512 > $O/L32_strong.json 2> $O/L32_strong.err || { echo L32_FAIL; tail -20 $O/L32_strong.err; exit 1; }
echo ALL_OK
