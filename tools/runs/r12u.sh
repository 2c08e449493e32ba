set -u
O=gpurun_out/r12u; mkdir -p $O
run() { local lim=$1 log=$2; shift 2; echo "== $log: $*"; timeout -k 10 $lim "$@" > $O/$log.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -30 $O/$log.log; exit $rc; fi; }
run 900 pytest python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread
tail -2 $O/pytest.log
run 300 smoke python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run 400 bench_c4 python3 -u bench.py
run 600 bench_c5 python3 -u bench.py --workload c5 --steps 2 --warmup 1 --no-cpu
grep -h '^{' $O/bench_c*.log | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); r=d['roofline']; print(d['config']['workload'], d['ms_per_step'], d['value'], r['v_write_ms'], r['v_read_ms'], r['h_read_ms'], r['frac'], r['traffic'])"
run 300 profc4 rocprofv3 --kernel-trace --stats --output-format csv -d $O/profc4 -o run -- python3 bench.py --no-cpu --steps 5 --warmup 2
run 400 shard python3 -u tools/shard_frame_bench.py --world 8 --rank 1 --reps 12 --rounds 3 --variants 0,134217728
grep '^{' $O/shard.log | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['variant'], d['ms_per_shard_frame_no_collective'])"
run 300 profshard rocprofv3 --kernel-trace --stats --output-format csv -d $O/profshard -o run -- python3 tools/shard_frame_bench.py --world 8 --rank 1 --reps 5
run 450 reh8 bash tools/rehearsal.sh $O 8
run 300 bench_wtaf python3 -u bench.py --no-cpu --flags 256
grep -h '^{' $O/bench_wtaf.log $O/bench_c4.log | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); r=d['roofline']; print(d['config']['api'], d['ms_per_step'], r.get('h_read_ms'), r.get('h_read_wta_scan_ms'))"
