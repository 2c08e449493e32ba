set -u
export TMPDIR=/tmp
# round-6 PMC of the 8-way C4 shard frame (every counter set; FETCH_SIZE / WRITE_SIZE
# for profiles/traffic.json c4_n8)
bash tools/gpu.sh r15d "pmcpy:tools/shard_frame_bench.py+--world+8+--rank+1+--reps+3"
