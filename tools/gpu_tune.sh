#!/bin/bash
# GPU session for kernel tuning: parity tests, pass microbenchmark over variants,
# then a counter pass on the default variant.  usage: tools/gpu_tune.sh TAG
set -u
TAG=${1:-tune}
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -rf -x > "$OUT/pytest_gpu_$TAG.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/pytest_gpu_$TAG.log"; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python tools/pass_bench.py --reps 8 ${VARIANTS:+--variants $VARIANTS} > "$OUT/pass_bench_$TAG.log" 2>&1
rc=$?; echo "pass_bench rc=$rc"; cat "$OUT/pass_bench_$TAG.log" | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
exit 0
