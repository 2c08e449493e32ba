set -u
export TMPDIR=/tmp
# C5 k_hpass11 den-read: cost prefetch depth, den ring depth, segment length
bash tools/gpu.sh r15j "cmd:python3 -u tools/exp/hpx_bench.py --c5 --reps 10 --forms 0,4,5,6,7,8,4,0"
