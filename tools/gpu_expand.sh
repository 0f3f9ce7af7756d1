# GPU box: two-wide expansion in the batched insert -- tests, build probe, bench graph quality
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/expand
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_screen.py tests/test_gpu_parity.py -k "batch or screen" > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
BUILD_BENCH=1 BUILD_OPTS="time_build=1,build_expand=1;time_build=1,build_expand=2" timeout -k 10 300 python -u tools/build_probe.py 400 > $O/probe.txt 2>&1 || { echo PROBE_FAIL; tail -20 $O/probe.txt; exit 1; }
BUILD_OPTS="build_expand=1;build_expand=2" timeout -k 10 300 python -u tools/build_probe.py 200 64 >> $O/probe.txt 2>&1 || { echo PROBE2_FAIL; tail -20 $O/probe.txt; exit 1; }
grep "^efc" $O/probe.txt
timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 --cpu-seconds 0 --no-shard-leg --build-expand 2 --ef-sweep 48,56,64,72 > $O/bench2.json 2> $O/bench2.err || { echo BENCH_FAIL; tail -20 $O/bench2.err; exit 1; }
python -c "import json; b=json.load(open('$O/bench2.json')); print(b['value'], b['recall_at_10'], b['build']['inserts_per_s'], [(p['ef'], p['recall_at_10'], p['qps']) for p in b['operating_points']])"
echo ALL_OK
