set -u
export TMPDIR=/tmp
# k_vpass32 with the left weights by DPP rows (DL) against the shipped form, alone and under rocprofv3
bash tools/gpu.sh r15h "cmd:python3 -u tools/exp/hs_bench.py --reps 60 --forms dl,full,prod,dl,full" \
  "profpy:tools/exp/hs_bench.py+--reps+10+--forms+full,dl"
