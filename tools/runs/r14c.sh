set -u
export TMPDIR=/tmp
# closing measurements of the round-6 tree: C4 bench (with the CPU baseline) and its
# kernel stats, PMC traffic of the C4 frame (c4_n1), the full counter sets of the passes,
# C5, the 8-way shard frame and its kernel stats, an 8-rank rehearsal
bash tools/gpu.sh r14c bench prof traffic pmc:--den "bench:--workload+c5+--steps+2+--warmup+1+--no-cpu" \
  "profpy:tools/shard_frame_bench.py+--world+8+--rank+1+--reps+5" \
  "cmd:python3 -u tools/shard_frame_bench.py --world 8 --rank 1 --reps 10 --rounds 3" \
  "cmd:bash tools/rehearsal.sh gpurun_out/r14c 8"
