set -u
O=gpurun_out/r12o; mkdir -p $O
run() { local lim=$1 log=$2; shift 2; echo "== $log: $*"; timeout -k 10 $lim "$@" > $O/$log.log 2>&1; local rc=$?; echo "   rc=$rc"; if [ $rc -ne 0 ]; then tail -30 $O/$log.log; exit $rc; fi; }
run 600 pytest_dl python3 -u -m pytest tests/test_gpu_pass32.py -m gpu -x -q --timeout 240 --timeout-method thread -k "dl_bit_exact or c4_shard or h_variants"
tail -2 $O/pytest_dl.log
run 300 passdl python3 -u tools/pass_bench.py --planes 32 --variants 0,134217728 --reps 10
grep '^{' $O/passdl.log
run 300 sharddl python3 -u tools/shard_frame_bench.py --world 8 --rank 1 --reps 10 --rounds 2 --variants 0,134217728
grep '^{' $O/sharddl.log
run 300 profdl rocprofv3 --kernel-trace --stats --output-format csv -d $O/profdl -o run -- python3 tools/shard_frame_bench.py --world 8 --rank 1 --reps 5 --variants 134217728
