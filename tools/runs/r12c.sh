set -u
O=gpurun_out/r12c; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "pass32 or wta_variants or test_support or abi" > $O/pytest_sel.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_sel.log; exit 1; }
tail -2 $O/pytest_sel.log
timeout -k 10 300 python3 -u tools/pass_bench.py --planes 32 --reps 10 --variants 0,67108864,134217728,201326592 > $O/pass32.log 2>&1 || { echo PASS_FAIL; tail -20 $O/pass32.log; exit 1; }
cat $O/pass32.log | grep '^{'
timeout -k 10 300 python3 -u tools/shard_frame_bench.py --world 8 --rank 1 --reps 10 --variants 0,67108864,134217728,201326592 --rounds 3 > $O/shard.log 2>&1 || { echo SHARD_FAIL; tail -20 $O/shard.log; exit 1; }
cat $O/shard.log | grep '^{'
timeout -k 10 300 python3 -u tools/exp/exp_forms.py > $O/exp_forms.log 2>&1 || { echo FORMS_FAIL; tail -20 $O/exp_forms.log; exit 1; }
cat $O/exp_forms.log | grep '^{'
