#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel-trace summary.
# Each GPU step has its own time limit; any crash / timeout / fault ends the script.
# usage: tools/gpu_check.sh [tag] [steps]
set -u
TAG=${1:-r01}
STEPS=${2:-10}
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp

stop_on_crash() {  # $1 = exit code, $2 = step name
    case "$1" in
        0|1) return 0 ;;  # 1 = test failures (no crash): keep going
        *) echo "STEP $2 ended with $1: stopping" | tee -a "$OUT/steps.log"; exit "$1" ;;
    esac
}

echo "== pytest -m gpu" | tee "$OUT/steps.log"
timeout -k 10 1200 python -m pytest tests -m gpu -q -rf > "$OUT/pytest_gpu_$TAG.log" 2>&1
rc=$?; echo "pytest rc=$rc" | tee -a "$OUT/steps.log"; tail -15 "$OUT/pytest_gpu_$TAG.log"; stop_on_crash $rc pytest

echo "== smoke" | tee -a "$OUT/steps.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
rc=$?; echo "smoke rc=$rc" | tee -a "$OUT/steps.log"; tail -3 "$OUT/smoke_$TAG.log"; [ $rc -eq 0 ] || exit $rc

echo "== bench" | tee -a "$OUT/steps.log"
timeout -k 10 600 python bench.py --steps "$STEPS" --warmup 2 > "$OUT/bench_$TAG.log" 2>&1
rc=$?; echo "bench rc=$rc" | tee -a "$OUT/steps.log"; tail -3 "$OUT/bench_$TAG.log"; [ $rc -eq 0 ] || exit $rc

echo "== rocprofv3 kernel trace" | tee -a "$OUT/steps.log"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o run -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu > "$OUT/prof_$TAG.log" 2>&1
rc=$?; echo "rocprof rc=$rc" | tee -a "$OUT/steps.log"; tail -3 "$OUT/prof_$TAG.log"; [ $rc -eq 0 ] || exit $rc
find "$OUT/prof_$TAG" -name "*stats*" | head

# HBM traffic counters, one counter per pass (FETCH_SIZE and WRITE_SIZE do not fit together)
for c in FETCH_SIZE WRITE_SIZE; do
  echo "== rocprofv3 --pmc $c" | tee -a "$OUT/steps.log"
  timeout -k 10 600 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$TAG/$c" -o run -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu > "$OUT/pmc_${TAG}_$c.log" 2>&1
  rc=$?; echo "pmc $c rc=$rc" | tee -a "$OUT/steps.log"; [ $rc -eq 0 ] || { tail -5 "$OUT/pmc_${TAG}_$c.log"; exit $rc; }
done
exit 0
