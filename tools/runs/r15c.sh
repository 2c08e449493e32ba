set -u
export TMPDIR=/tmp
# closing validation of the round-6 tree (library rebuilt after the HS template change,
# product ISA unchanged): smoke, the whole GPU suite, the C4 bench with its CPU baseline
# and kernel stats, the 8-way shard frame
bash tools/gpu.sh r15c smoke test bench prof \
  "cmd:python3 -u tools/shard_frame_bench.py --world 8 --rank 1 --reps 10 --rounds 3"
