set -u
export TMPDIR=/tmp
# final tree (nt stores in k_support / k_raw_cost): smoke and the whole GPU suite
bash tools/gpu.sh r15p smoke test
