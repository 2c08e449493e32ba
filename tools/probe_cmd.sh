set -e
mkdir -p gpurun_out/r05d
for n in 0 1 2 3 4 8 15; do
  echo "probe $n" >> gpurun_out/r05d/probe.log
  ASW_LIB=stereo_matchin_amd/libasw_probe$n.so timeout -k 10 120 python3 tools/pass_bench.py --reps 6 --den --variants 0 2>/dev/null | grep '"v"' >> gpurun_out/r05d/probe.log
done
cat gpurun_out/r05d/probe.log
