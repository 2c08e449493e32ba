set -u
export TMPDIR=/tmp
# C5 den-read H pass with PX = 24 shipped: the C5 parity tests, the C5 bench, the whole
# GPU suite, the C4 bench
bash tools/gpu.sh r15k "test:c5" "bench:--workload+c5+--steps+2+--warmup+1+--no-cpu" test "bench:--no-cpu"
