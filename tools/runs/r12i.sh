set -u
O=gpurun_out/r12i; mkdir -p $O
run() { local lim=$1 log=$2; shift 2; echo "== $log: $*"; timeout -k 10 $lim "$@" > $O/$log.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -30 $O/$log.log; exit $rc; fi; }
run 600 vtile_c4 python3 -u tools/exp/exp_bench.py --v --lib none --reps 8 --vexps prod_read,vtile1,vtile2,vtile4,vtile8
grep '^{\|error' $O/vtile_c4.log
run 900 vtile_c5 python3 -u tools/exp/exp_bench.py --c5 --v --lib none --reps 3 --vexps prod_read,vtile4,vtile8,vtile2
grep '^{\|error' $O/vtile_c5.log
