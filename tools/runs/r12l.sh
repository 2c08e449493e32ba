set -u
O=gpurun_out/r12l; mkdir -p $O
run() { local lim=$1 log=$2; shift 2; echo "== $log: $*"; timeout -k 10 $lim "$@" > $O/$log.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -30 $O/$log.log; exit $rc; fi; }
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  run 300 pmc_c4_$c rocprofv3 --pmc $c --output-format csv -d $O/pmc_c4/$c -o run -- python3 tools/exp/exp_bench.py --v --lib none --reps 2 --vexps prod_read,vtile4
done
for c in FETCH_SIZE WRITE_SIZE; do
  run 600 pmc_c5_$c rocprofv3 --pmc $c --output-format csv -d $O/pmc_c5/$c -o run -- python3 tools/exp/exp_bench.py --c5 --v --lib none --reps 1 --vexps prod_read,vtile4
done
