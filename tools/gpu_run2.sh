# quick GPU check: parity tests touching the pass / frame path, then the bench and a kernel trace
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_r2.log 2>&1
rc=$?; tail -3 gpurun_out/pt_r2.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_r2.log 2>&1
rc=$?; tail -1 gpurun_out/bench_r2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r2 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/prof_r2.log 2>&1
exit $?
