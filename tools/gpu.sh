#!/bin/bash
# One GPU-box session, parameterised by steps (replaces the round-1 one-off scripts).
#   tools/gpu.sh TAG step [step ...]
# steps:
#   test        pytest -m gpu (whole suite)           test:EXPR  only tests matching -k EXPR
#   smoke       __graft_entry__.smoke()
#   bench       python bench.py (default workload, with cpu_baseline)
#   bench:ARGS  python bench.py ARGS  ('+'-separated, e.g. bench:--workload+c5+--steps+3)
#   prof        rocprofv3 --kernel-trace --stats of bench.py --no-cpu
#   prof:ARGS   the same with bench.py ARGS
#   profpy:ARGS rocprofv3 --kernel-trace --stats of python3 ARGS (a tool script)
#   pass        tools/pass_bench.py (den modes, default variant)
#   pmc         rocprofv3 --pmc counter sets (one run each) over tools/pass_bench.py
#   pmcpy:ARGS  the same counter sets over python3 ARGS (e.g. tools/shard_frame_bench.py+--world+8)
#   calib       rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE over tools/ubench/fetch_calib
#   traffic     rocprofv3 --pmc FETCH_SIZE, then WRITE_SIZE, over bench.py (C4 frame) -> $OUT/traffic
#   cmd:STR     any other command (STR runs under bash with a 300 s limit)
# Every GPU step runs under its own `timeout -k 10`; the first step that fails
# (non-zero exit, crash, time limit) ends the script with its status.
set -u
TAG=${1:?tag}
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
PY="python3 -u"

run() {  # $1 = seconds, $2 = log name, rest = command
    local lim=$1 log=$2
    shift 2
    echo "== [$log] $*" | tee -a "$OUT/steps.log"
    timeout -k 10 "$lim" "$@" > "$OUT/$log.log" 2>&1
    local rc=$?
    echo "   rc=$rc" | tee -a "$OUT/steps.log"
    tail -4 "$OUT/$log.log" | grep -v amdgpu.ids
    if [ $rc -ne 0 ]; then
        tail -30 "$OUT/$log.log"
        exit $rc
    fi
}

PMC_SETS=(
    "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES"
    "SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
    "SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_LDS SQ_INST_LEVEL_SMEM SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH SQ_IFETCH"
    "GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum"
    "FETCH_SIZE"
    "WRITE_SIZE"
)

for step in "$@"; do
    name=${step%%:*}
    arg=""
    [ "$name" != "$step" ] && arg=${step#*:}
    args=${arg//+/ }
    case "$name" in
        test)
            if [ -n "$arg" ]; then
                run 900 "pytest_$TAG" $PY -m pytest tests -m gpu -x -v -k "$args" --timeout 240 --timeout-method thread
            else
                run 1100 "pytest_$TAG" $PY -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread
            fi ;;
        smoke) run 300 "smoke_$TAG" $PY -c "import __graft_entry__ as g; g.smoke()" ;;
        bench) run 600 "bench_$TAG${arg:+_${args// /_}}" $PY bench.py $args ;;
        prof)
            run 600 "prof_$TAG" rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
                python3 bench.py --steps 5 --warmup 1 --no-cpu $args ;;
        profpy)  # rocprofv3 kernel stats of any python script: profpy:tools/x.py+--arg+v
            nprof=$((${nprof:-0} + 1))
            run 600 "profpy${nprof}_$TAG" rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profpy$nprof" -o run -- \
                python3 $args ;;
        pass) run 600 "pass_$TAG${arg:+_${args// /_}}" $PY tools/pass_bench.py --reps 6 --den ${args:---variants 0} ;;
        pmc)
            i=0
            for set in "${PMC_SETS[@]}"; do
                i=$((i + 1))
                run 300 "pmc_$TAG$i" rocprofv3 --pmc $set --output-format csv -d "$OUT/pmc/p$i" -o run -- \
                    python3 tools/pass_bench.py --reps 1 --den ${args:---variants 0}
            done ;;
        pmcpy)  # every counter set over any python script: pmcpy:tools/x.py+--arg+v -> $OUT/pmcpy/p<i>
            i=0
            for set in "${PMC_SETS[@]}"; do
                i=$((i + 1))
                run 300 "pmcpy_$TAG$i" rocprofv3 --pmc $set --output-format csv -d "$OUT/pmcpy/p$i" -o run -- \
                    python3 $args
            done ;;
        calib)
            for c in FETCH_SIZE WRITE_SIZE; do
                run 120 "calib_$c" rocprofv3 --pmc $c --output-format csv -d "$OUT/calib/$c" -o run -- \
                    tools/ubench/fetch_calib
            done ;;
        traffic)
            i=0
            for c in FETCH_SIZE WRITE_SIZE; do
                i=$((i + 1))
                run 300 "traffic_$c" rocprofv3 --pmc $c --output-format csv -d "$OUT/traffic/p$i" -o run -- \
                    python3 bench.py --steps 2 --warmup 1 --no-cpu $args
            done ;;
        cmd) ncmd=$((${ncmd:-0} + 1)); run 300 "cmd${ncmd}_$TAG" bash -c "$arg" ;;
        *) echo "unknown step $step"; exit 2 ;;
    esac
done
exit 0
