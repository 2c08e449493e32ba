#!/bin/bash
# Counter collection for the aggregation passes (separate --pmc passes, no tracing
# domains mixed in).  usage: tools/gpu_pmc.sh TAG [variant]
set -u
TAG=${1:-pmc}
VAR=${2:-0}
OUT=gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
CMD="python3 tools/pass_bench.py --reps 2 --variants $VAR"
i=0
SETS=${SETS:-all}
if [ "$SETS" = "lat" ]; then LIST=(
  "SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
  "SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_ACTIVE_INST_VALU"
  "GRBM_GUI_ACTIVE SQ_LEVEL_WAVES SQ_WAVES SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM" )
elif [ "$SETS" = "icache" ]; then LIST=(
  "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_WAVE_CYCLES"
  "SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_SALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" )
else LIST=(
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES" \
  "SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" \
  "GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum" \
  "FETCH_SIZE" \
  "WRITE_SIZE" ); fi
for set in "${LIST[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d "$OUT/p$i" -o run -- $CMD > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pmc set $i rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$OUT/p$i.log"; exit $rc; }
done
exit 0
