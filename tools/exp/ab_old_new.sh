#!/bin/bash
# A/B of the committed library (tools/exp/libasw_old.so, DEV build of the previous tree)
# against the working tree's library on one box: C4 bench lines + kernel stats.
set -e
O=gpurun_out/$1; mkdir -p $O
for i in 1 2; do
  ASW_LIB=tools/exp/libasw_old.so timeout -k 10 200 python3 -u bench.py --no-cpu --steps 20 > $O/old_$i.json 2>/dev/null
  timeout -k 10 200 python3 -u bench.py --no-cpu --steps 20 > $O/new_$i.json 2>/dev/null
done
ASW_LIB=tools/exp/libasw_old.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_old -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu > /dev/null 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_new -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu > /dev/null 2>&1
for f in $O/old_*.json $O/new_*.json; do python3 -c "import json,sys; d=json.load(open('$f')); r=d['roofline']; print('$f', d['ms_per_step'], r['v_read_ms'], r['h_read_ms'], r['v_write_ms'], r['h_write_ms'])"; done
