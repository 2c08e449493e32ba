#!/bin/bash
# k_support with the LUT in LDS (tools/exp/libasw_sl.so, DEV build with ASW_SUPPORT_LDS=1)
# against the production library: parity (support tests) and C4 kernel stats
set -e
O=gpurun_out/$1; mkdir -p $O
ASW_LIB=tools/exp/libasw_sl.so timeout -k 10 300 python3 -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "support" --timeout 120 > $O/pytest_sl.log 2>&1 || { tail -20 $O/pytest_sl.log; exit 1; }
tail -1 $O/pytest_sl.log
for v in prod sl prod sl; do
  if [ $v = prod ]; then L=""; else L=tools/exp/libasw_$v.so; fi
  ASW_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu > /dev/null 2>&1
  python3 -c "import csv; [print(\"$v\", r[\"Name\"][:40], r[\"Calls\"], float(r[\"AverageNs\"])/1e6) for r in csv.DictReader(open(\"$O/$v/run_kernel_stats.csv\")) if \"k_support\" in r[\"Name\"]]"
done
