set -u
O=gpurun_out/r12k; mkdir -p $O
run() { local lim=$1 log=$2; shift 2; echo "== $log: $*"; timeout -k 10 $lim "$@" > $O/$log.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -30 $O/$log.log; exit $rc; fi; }
run 600 pytest_pipe python3 -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -q --timeout 240 --timeout-method thread
tail -2 $O/pytest_pipe.log
run 300 shard_pipe python3 -u tools/shard_frame_bench.py --world 8 --rank 1 --reps 10 --rounds 3 --pipeline 0,1
grep '^{' $O/shard_pipe.log
run 300 bench_plain python3 -u bench.py --no-cpu --pipeline off
run 300 bench_pipe0 python3 -u bench.py --no-cpu --pipeline on --overlap-prep 0
run 300 bench_pipe1 python3 -u bench.py --no-cpu --pipeline on --overlap-prep 1
run 300 bench_plain_b python3 -u bench.py --no-cpu --pipeline off
run 300 bench_pipe1_b python3 -u bench.py --no-cpu --pipeline on --overlap-prep 1
grep -h '^{' $O/bench_*.log | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['config']['api'], d['ms_per_step'], d['value'])"
