set -u
O=gpurun_out/r14d; mkdir -p $O
export TMPDIR=/tmp
run() { local lim=$1 log=$2; shift 2; echo "== $log: $*"; timeout -k 10 $lim "$@" > $O/$log.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -30 $O/$log.log; exit $rc; fi; }
run 300 vprobe python3 -u tools/exp/exp_bench.py --lib none --reps 8 --vprobe 0:0,0:128,1:128,2:0,2:128,2:8,2:4,2:79
grep '^{' $O/vprobe.log
