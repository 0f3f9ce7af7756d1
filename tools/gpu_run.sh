#!/bin/bash
# The one GPU-box runner (through gpurun).  Steps run in order, each under its
# own time limit; the first failing step ends the run (no retries, nothing
# after a fault), and every step's output lands in gpurun_out/TAG/.
#
#   bash tools/gpu_run.sh TAG STEP [STEP ...]
#     smoke              __graft_entry__.smoke()
#     suite              the whole GPU suite (pytest -m gpu)
#     test:A,B,...       pytest -m gpu with the arguments A B ... (paths, -k EXPR)
#     bench[:A,B,...]    bench.py (the driver's command: --gpus 1 --steps 20 --warmup 5) plus A B ...
#     rehearse2          the driver's N=2 command as 2 gloo ranks on this one GPU
#     prof[:A,B,...]     tools/profile_round.sh TAG (kernel trace + FETCH/WRITE PMC) with A B ...
#     py:SCRIPT[,A,...]  python SCRIPT A ... (a tools/ probe)
#     pyl:LIB,SCRIPT[,A,...]  the same on tools/LIB (a tools/Makefile.beam variant; push it: take it out of .gpurunignore)
#     gemm:T,...         tools/gemm_diag.sh T ... (configs[4] exact path, rocprofv3 stats per exact_tile T)
#     diag:T,...         the same on tools/libmhnsw_diag.so (timing-diagnostic variants; needs the .so
#                        pushed: take ./tools/libmhnsw_*.so out of .gpurunignore for that call)
#     yard               rocprofv3 stats of tools/gemm_yardstick.py (torch fp16 matmul, configs[4] shape)
#     cprof              compat Add cycle accounting (tools/libmhnsw_cprof.so, tools/cprof_probe.py + cprof_sum.py)
set -o pipefail
TAG=$1
shift
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$TAG
mkdir -p "$O"
PYT="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu"
i=0
for step in "$@"; do
    i=$((i + 1))
    name=${step%%:*}
    args=""
    [[ "$step" == *:* ]] && args=${step#*:} && args=${args//,/ }
    log=$O/$i.$name.log
    echo "[$i] $step" >&2
    case "$name" in
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$log" 2>&1 ;;
    suite) timeout -k 10 1100 $PYT tests > "$log" 2>&1 ;;
    test) timeout -k 10 900 $PYT $args > "$log" 2>&1 ;;
    bench) timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 $args > "$O/$i.bench.json" 2> "$log" ;;
    rehearse2) timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --one-gpu \
        --backend gloo $args > "$O/$i.rehearse2.json" 2> "$log" ;;
    prof) timeout -k 10 1100 bash tools/profile_round.sh "$TAG/prof$i" $args > "$log" 2>&1 ;;
    py) timeout -k 10 900 python -u $args > "$log" 2>&1 ;;
    pyl) set -- $args && lib=$1 && shift &&
        MHNSW_LIB=$PWD/tools/$lib timeout -k 10 900 python -u "$@" > "$log" 2>&1 ;;
    gemm) timeout -k 10 900 bash tools/gemm_diag.sh $args > "$log" 2>&1 ;;
    diag) MHNSW_LIB=$PWD/tools/libmhnsw_diag.so timeout -k 10 900 bash tools/gemm_diag.sh $args > "$log" 2>&1 ;;
    cprof) MHNSW_LIB=$PWD/tools/libmhnsw_cprof.so timeout -k 10 600 python -u tools/cprof_probe.py > "$log" 2>&1 &&
        python tools/cprof_sum.py "$log" > "$O/$i.cprof_sum.txt" ;;
    yard) (cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/yard" \
        -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/gemm_yardstick.py" 20) > "$log" 2>&1 ;;
    *) echo "unknown step $step" >&2; exit 8 ;;
    esac
    rc=$?
    if [ $rc -ne 0 ]; then
        echo "FAIL step $i ($step) rc=$rc"
        tail -40 "$log"
        exit 1
    fi
    tail -3 "$log"
done
echo ALL_OK
