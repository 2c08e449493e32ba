set -u
export TMPDIR=/tmp
# nontemporal stores in k_support / k_raw_cost: GPU tests of those kernels, C4 bench A/B
# against the previous library on one box (ASW_LIB), kernel stats
B="python3 -u bench.py --no-cpu --steps 30"
bash tools/gpu.sh r15o "test:support+or+raw" "cmd:$B" "cmd:ASW_LIB=tools/exp/libasw_prev.so $B" "cmd:$B" \
  "cmd:ASW_LIB=tools/exp/libasw_prev.so $B" prof "cmd:python3 -u tools/shard_frame_bench.py --world 8 --rank 1 --reps 10 --rounds 3" \
  "cmd:ASW_LIB=tools/exp/libasw_prev.so python3 -u tools/shard_frame_bench.py --world 8 --rank 1 --reps 10 --rounds 3"
