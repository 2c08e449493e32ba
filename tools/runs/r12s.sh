set -u
O=gpurun_out/r12s; mkdir -p $O
run() { local lim=$1 log=$2; shift 2; echo "== $log: $*"; timeout -k 10 $lim "$@" > $O/$log.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -30 $O/$log.log; exit $rc; fi; }
run 600 pytest_sup python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pass32.py tests/test_gpu_frame.py -m gpu -x -q --timeout 240 --timeout-method thread -k "support or raw or e2e or c4_full or shard_band or frame"
tail -2 $O/pytest_sup.log
run 300 profc4 rocprofv3 --kernel-trace --stats --output-format csv -d $O/profc4 -o run -- python3 bench.py --no-cpu --steps 5 --warmup 2
run 300 profshard rocprofv3 --kernel-trace --stats --output-format csv -d $O/profshard -o run -- python3 tools/shard_frame_bench.py --world 8 --rank 1 --reps 5
for f in profc4 profshard; do grep -h "k_support\|k_raw" $O/$f/run_kernel_stats.csv | cut -d, -f1,2,4 | cut -c1-40,150-; done
run 300 shard python3 -u tools/shard_frame_bench.py --world 8 --rank 1 --reps 12 --rounds 3
grep '^{' $O/shard.log | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['variant'], d['ms_per_shard_frame_no_collective'])"
