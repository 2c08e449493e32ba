#!/bin/bash
# k_wta_scan diagnostics: kernel stats of the C4 bench with the production library and
# the ASW_WTA_PROBE builds (1: coalesced target reads, 2: no target reads; WRONG results)
set -e
O=gpurun_out/$1; mkdir -p $O
for v in ${VARIANTS:-prod wp1 wp2}; do
  if [ $v = prod ]; then L=""; else L=tools/exp/libasw_$v.so; fi
  ASW_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu > /dev/null 2>&1
  python3 -c "import csv; [print(\"$v\", r[\"Calls\"], float(r[\"AverageNs\"])/1e6) for r in csv.DictReader(open(\"$O/$v/run_kernel_stats.csv\")) if \"k_wta_scan\" in r[\"Name\"]]"
done
