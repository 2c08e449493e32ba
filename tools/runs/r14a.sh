set -u
O=gpurun_out/r14a; mkdir -p $O
export TMPDIR=/tmp
run() { local lim=$1 log=$2; shift 2; echo "== $log: $*"; timeout -k 10 $lim "$@" > $O/$log.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -30 $O/$log.log; exit $rc; fi; }
run 300 smoke python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run 300 vdma python3 -u tools/exp/exp_bench.py --lib none --vdma 64 --reps 8
grep '^{' $O/vdma.log
run 300 vprobe python3 -u tools/exp/exp_bench.py --lib none --reps 6 --vprobe 0:0,0:3,0:15,0:16,0:32,0:47,0:19,0:8,2:0,2:67,2:16,2:32,kd:4,kd:5,kd:8
grep '^{' $O/vprobe.log
run 400 bench_c4 python3 -u bench.py
grep '^{' $O/bench_c4.log | cut -c1-600
run 300 profc4 rocprofv3 --kernel-trace --stats --output-format csv -d $O/profc4 -o run -- python3 bench.py --no-cpu --steps 5 --warmup 2
run 900 pytest python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread
tail -2 $O/pytest.log
