set -u
O=gpurun_out/r12p; mkdir -p $O
run() { local lim=$1 log=$2; shift 2; echo "== $log: $*"; timeout -k 10 $lim "$@" > $O/$log.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -30 $O/$log.log; exit $rc; fi; }
run 600 pytest_raw python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pass32.py -m gpu -x -q --timeout 240 --timeout-method thread -k "raw or c4_shard or h_variants or pass32_bit_exact or dl_bit_exact"
tail -2 $O/pytest_raw.log
V=0,5242880,6291456,134217728,139460608,140509184,167772160,173015040,174063616
run 300 passdl python3 -u tools/pass_bench.py --planes 32 --variants $V --reps 10
grep '^{' $O/passdl.log | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l)
    if d['dir'] in ('v','h'): print(d['variant'], d['dir'], d['ms_median'], d['ms_min'])"
run 300 sharddl python3 -u tools/shard_frame_bench.py --world 8 --rank 1 --reps 10 --rounds 2 --variants 0,139460608,140509184,173015040,174063616,134217728
grep '^{' $O/sharddl.log | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['variant'], d['ms_per_shard_frame_no_collective'])"
run 300 profc4 rocprofv3 --kernel-trace --stats --output-format csv -d $O/profc4 -o run -- python3 bench.py --no-cpu --steps 5 --warmup 2
head -12 $O/profc4/run_kernel_stats.csv | cut -c1-60,200-260
