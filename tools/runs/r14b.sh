set -u
O=gpurun_out/r14b; mkdir -p $O
export TMPDIR=/tmp
run() { local lim=$1 log=$2; shift 2; echo "== $log: $*"; timeout -k 10 $lim "$@" > $O/$log.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -30 $O/$log.log; exit $rc; fi; }
ls -la stereo_matchin_amd/libasw_hip.so
run 300 smoke python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run 300 hwta python3 -u tools/exp/exp_bench.py --lib none --hwta 0,1 --reps 8
grep '^{' $O/hwta.log
run 400 bench_c4 python3 -u bench.py --no-cpu
grep '^{' $O/bench_c4.log | cut -c1-400
run 900 pytest python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread
tail -2 $O/pytest.log
