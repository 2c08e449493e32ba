set -u
export TMPDIR=/tmp
# k_hpass32 PX = 8 shipped for T = 35: the 32-plane tests, the shard frame A/B against
# the previous library on one box (ASW_LIB), then the whole GPU suite
SB="python3 -u tools/shard_frame_bench.py --world 8 --rank 1 --reps 10 --rounds 3"
bash tools/gpu.sh r15g "test:pass32+or+shard" \
  "cmd:$SB" "cmd:ASW_LIB=tools/exp/libasw_prev.so $SB" "cmd:$SB" "cmd:ASW_LIB=tools/exp/libasw_prev.so $SB" \
  "profpy:tools/shard_frame_bench.py+--world+8+--rank+1+--reps+5" test
