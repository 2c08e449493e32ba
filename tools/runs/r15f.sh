set -u
export TMPDIR=/tmp
# k_hpass32 with a deeper cost prefetch (exp forms 4: PX 8, 5: PX 16) against the shipped form
bash tools/gpu.sh r15f "cmd:python3 -u tools/exp/h32_bench.py --reps 60 --runs 4:0,0:0,4:6,0:6,5:0"
