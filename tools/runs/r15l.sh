set -u
export TMPDIR=/tmp
# C5 V den-read: one barrier per row (no spills) and a deeper prefetch, against the shipped form
bash tools/gpu.sh r15l "cmd:python3 -u tools/exp/c5v_bench.py --reps 8 --forms 2,1,81,2,1,81"
