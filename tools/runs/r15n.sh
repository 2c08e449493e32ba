set -u
export TMPDIR=/tmp
# closing run of the final tree: smoke, the C4 bench with its CPU baseline and kernel
# stats, the 8-way shard frame and its kernel stats
bash tools/gpu.sh r15n smoke bench prof \
  "cmd:python3 -u tools/shard_frame_bench.py --world 8 --rank 1 --reps 10 --rounds 3" \
  "profpy:tools/shard_frame_bench.py+--world+8+--rank+1+--reps+5"
