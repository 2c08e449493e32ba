set -u
O=gpurun_out/r12t; mkdir -p $O
run() { local lim=$1 log=$2; shift 2; echo "== $log: $*"; timeout -k 10 $lim "$@" > $O/$log.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -30 $O/$log.log; exit $rc; fi; }




run 300 bench_f1 python3 -u bench.py --no-cpu
run 300 bench_f0 python3 -u bench.py --no-cpu --wta-fused 0
run 300 bench_f1b python3 -u bench.py --no-cpu
run 300 bench_f0b python3 -u bench.py --no-cpu --wta-fused 0
run 300 bench_frame python3 -u bench.py --no-cpu --api frame
grep -h '^{' $O/bench_*.log | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); r=d['roofline']; print(d['config']['api'], d['ms_per_step'], r.get('h_read_ms'), r.get('h_read_wta_scan_ms'))"
run 300 profc4 rocprofv3 --kernel-trace --stats --output-format csv -d $O/profc4 -o run -- python3 bench.py --no-cpu --steps 5 --warmup 2
head -14 $O/profc4/run_kernel_stats.csv | cut -d, -f1,2,4 | cut -c1-60,150-
