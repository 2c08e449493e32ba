#!/bin/bash
# A/B of the raw-cost / support overlap (stage API): C4 bench lines alternating
set -e
O=gpurun_out/$1; mkdir -p $O
for i in 1 2 3; do
  for m in serial overlap; do
    if [ $m = serial ]; then E=1; else E=0; fi
    ASW_SERIAL_RAW=$E timeout -k 10 200 python3 -u bench.py --no-cpu --steps 30 > $O/${m}_$i.json 2>/dev/null
    python3 -c "import json; d=json.load(open('$O/${m}_$i.json')); print('$m', d['ms_per_step'])"
  done
done
