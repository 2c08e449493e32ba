set -u
O=gpurun_out/r12q; mkdir -p $O
run() { local lim=$1 log=$2; shift 2; echo "== $log: $*"; timeout -k 10 $lim "$@" > $O/$log.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -30 $O/$log.log; exit $rc; fi; }
run 600 pytest_dl python3 -u -m pytest tests/test_gpu_pass32.py -m gpu -x -q --timeout 240 --timeout-method thread
tail -2 $O/pytest_dl.log
run 300 passdl python3 -u tools/pass_bench.py --planes 32 --variants 0,134217728 --reps 12
grep '^{' $O/passdl.log | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l)
    if d['dir'] in ('v','h'): print(d['variant'], d['dir'], d['ms_median'], d['ms_min'])"
run 400 sharddl python3 -u tools/shard_frame_bench.py --world 8 --rank 1 --reps 12 --rounds 4 --variants 0,134217728
grep '^{' $O/sharddl.log | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['variant'], d['ms_per_shard_frame_no_collective'])"
run 300 profdl rocprofv3 --kernel-trace --stats --output-format csv -d $O/profdl -o run -- python3 tools/shard_frame_bench.py --world 8 --rank 1 --reps 5 --variants 0,134217728
i=0
for c in FETCH_SIZE WRITE_SIZE; do
  i=$((i + 1))
  run 400 pmc5_$c rocprofv3 --pmc $c --output-format csv -d $O/pmc_c5/p$i -o run -- python3 bench.py --workload c5 --steps 1 --warmup 0 --no-cpu
done
