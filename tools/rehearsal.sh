#!/bin/bash
# bench.py's N > 1 path on a one-GPU box: N ranks on GPU 0, gloo collectives
# (ASW_BENCH_REHEARSAL=1; the numbers are not a scaling measurement).
#   tools/rehearsal.sh OUTDIR N [bench args ...]
set -e
O=$1; N=$2; shift 2
mkdir -p "$O"
ASW_BENCH_REHEARSAL=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" \
    --master-addr 127.0.0.1 --master-port $((29400 + RANDOM % 500)) bench.py --gpus "$N" --steps 2 --warmup 1 --no-cpu "$@" \
    > "$O/rehearsal$N${1:+_g}.log" 2>&1
grep '^{' "$O/rehearsal$N${1:+_g}.log"
