set -u
export TMPDIR=/tmp
# k_hpass11 den-read with a deeper cost prefetch: C4 and C5, bit-exact check + timing
bash tools/gpu.sh r15i "cmd:python3 -u tools/exp/hpx_bench.py --reps 40 --forms 10,11,10,11" \
  "cmd:python3 -u tools/exp/hpx_bench.py --c5 --reps 8 --forms 0,1,2,3,4"
