set -u
O=gpurun_out/r12n; mkdir -p $O
run() { local lim=$1 log=$2; shift 2; echo "== $log: $*"; timeout -k 10 $lim "$@" > $O/$log.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -30 $O/$log.log; exit $rc; fi; }
run 240 hybrid_v python3 -u tools/exp/hybrid_probe.py --dir v
run 240 hybrid_h python3 -u tools/exp/hybrid_probe.py --dir h
cat $O/hybrid_v.log $O/hybrid_h.log | grep '^{'
