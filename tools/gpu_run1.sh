set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "variants" --timeout 120 --timeout-method thread > gpurun_out/pt_v32.log 2>&1
rc=$?; tail -3 gpurun_out/pt_v32.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/pass_bench.py --reps 6 --variants 0,128,256 --den > gpurun_out/pb_v32.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/pb_v32.log; exit $rc
