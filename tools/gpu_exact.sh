# GPU box: exact-path parity tests, config-5 timings per precision / tile, kernel-trace stats
# and PMC passes of precision 3 (tile $1, default 1)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${1:-1}
O=$GRAFT_REPO_ROOT/gpurun_out/exact
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_screen.py -k "exact or screen" > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu tests/test_gpu_fullsize.py -k "c5" > $O/pytest_c5.log 2>&1 || { echo C5_FAIL; tail -40 $O/pytest_c5.log; exit 1; }
tail -1 $O/pytest_c5.log
timeout -k 10 400 python -u tools/bench_configs.py 5 5t > $O/cfg5.jsonl 2> $O/cfg5.err || { echo CFG5_FAIL; tail -20 $O/cfg5.err; exit 1; }
cat $O/cfg5.jsonl
cd /tmp && export TMPDIR=/tmp
P="python3 $GRAFT_REPO_ROOT/tools/exact_probe.py 3 $T 5"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $P > $O/trace.log 2>&1 || { echo TRACE_FAIL; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $O/sq -o run --output-format csv -- $P > $O/sq.log 2>&1 || { echo PMC1_FAIL; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/tcc -o run --output-format csv -- $P > $O/tcc.log 2>&1 || { echo PMC2_FAIL; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU -d $O/sq2 -o run --output-format csv -- $P > $O/sq2.log 2>&1 || { echo PMC3_FAIL; exit 1; }
echo ALL_OK
