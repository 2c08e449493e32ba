set -u
O=gpurun_out/r12h; mkdir -p $O
run() { local lim=$1 log=$2; shift 2; echo "== $log: $*"; timeout -k 10 $lim "$@" > $O/$log.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -30 $O/$log.log; exit $rc; fi; }
run 900 pytest python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread
tail -2 $O/pytest.log
run 300 bench_a python3 -u bench.py --no-cpu
run 300 bench_f32_a python3 -u bench.py --flags 64 --no-cpu
run 300 bench_b python3 -u bench.py --no-cpu
run 300 bench_f32_b python3 -u bench.py --flags 64 --no-cpu
grep -h '^{' $O/bench_*.log | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); r=d['roofline']; print(d['config']['flags'], d['ms_per_step'], r['v_write_ms'], r['v_read_ms'], r['h_read_ms'], r['kernels_ran'].get('V den-write'))"
run 300 shard python3 -u tools/shard_frame_bench.py --world 8 --rank 1 --reps 10 --flags 0,64,128 --rounds 3
grep '^{' $O/shard.log
run 300 profshard rocprofv3 --kernel-trace --stats --output-format csv -d $O/profshard -o run -- python3 tools/shard_frame_bench.py --world 8 --rank 1 --reps 5 --flags 0,128
run 600 bench_c5 python3 -u bench.py --workload c5 --steps 2 --warmup 1 --no-cpu
run 600 bench_c5_f32 python3 -u bench.py --workload c5 --steps 2 --warmup 1 --no-cpu --flags 64
grep -h '^{' $O/bench_c5*.log | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['config']['flags'], d['ms_per_step'], d['roofline']['v_write_ms'])"
