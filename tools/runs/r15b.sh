set -u
O=gpurun_out/r15b; mkdir -p $O
export TMPDIR=/tmp
run() { local lim=$1 log=$2; shift 2; echo "== $log: $*"; timeout -k 10 $lim "$@" > $O/$log.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -30 $O/$log.log; exit $rc; fi; }
run 300 hs python3 -u tools/exp/hs_bench.py --reps 30
cat $O/hs.log | grep -v Gloo
run 300 hsprof rocprofv3 --kernel-trace --stats --output-format csv -d $O/hsprof -o run -- python3 tools/exp/hs_bench.py --reps 10
