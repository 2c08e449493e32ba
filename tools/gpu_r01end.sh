# round-end check: gpu parity tests, smoke, default bench (with cpu_baseline), kernel trace
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_r01end.log 2>&1
rc=$?; tail -3 gpurun_out/pt_r01end.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r01end.log 2>&1
rc=$?; tail -2 gpurun_out/smoke_r01end.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_r01end.log 2>&1
rc=$?; tail -1 gpurun_out/bench_r01end.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r01end -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/prof_r01end.log 2>&1
exit $?
