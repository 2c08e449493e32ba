set -u
export TMPDIR=/tmp
# C5 den-write H pass with the deeper cost prefetch (bit-exact out and den)
bash tools/gpu.sh r15m "cmd:python3 -u tools/exp/hpx_bench.py --c5 --reps 8 --forms 20,21,22,20,21"
