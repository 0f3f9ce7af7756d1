# GPU box: expansion widths 2-4 in the batched insert -- tests, build probe, served-graph quality
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/expand4
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_screen.py tests/test_gpu_parity.py -k "batch or screen" > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
BUILD_BENCH=1 BUILD_OPTS="time_build=1,build_expand=2;time_build=1,build_expand=3;time_build=1,build_expand=4" timeout -k 10 300 python -u tools/build_probe.py 400 > $O/probe.txt 2>&1 || { echo PROBE_FAIL; tail -20 $O/probe.txt; exit 1; }
BUILD_OPTS="build_expand=2;build_expand=3;build_expand=4" timeout -k 10 300 python -u tools/build_probe.py 64 >> $O/probe.txt 2>&1 || { echo PROBE2_FAIL; tail -20 $O/probe.txt; exit 1; }
grep "^efc" $O/probe.txt
for X in 3 4; do
timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 --cpu-seconds 0 --no-shard-leg --configs '' --build-expand $X --ef-sweep 56,64,72 > $O/bench$X.json 2> $O/bench$X.err || { echo BENCH_FAIL; tail -20 $O/bench$X.err; exit 1; }
python -c "import json; b=json.load(open('$O/bench$X.json')); print($X, b['value'], b['recall_at_10'], b['build']['inserts_per_s'], [(p['ef'], p['recall_at_10'], p['qps']) for p in b['operating_points']])"
done
echo ALL_OK
