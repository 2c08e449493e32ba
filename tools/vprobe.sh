#!/bin/bash
# Builds diagnostic V-pass libraries (T = 35 only, ASW_VPROBE bits, see
# asw_aggregate_impl.h; their results are WRONG) for tools/pass_bench.py runs with
# ASW_LIB=stereo_matchin_amd/libasw_probe<N>.so.   tools/vprobe.sh 1 2 3 ...
set -e
cd "$(dirname "$0")/../stereo_matchin_amd/csrc"
for n in "$@"; do
    make -s -j8 DEV=1 B=build_probe$n OUT=../libasw_probe$n.so EXTRA="-DASW_DEV_TAPS=35 -DASW_VPROBE=$n"
done
