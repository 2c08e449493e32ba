#!/bin/bash
# kernel resource metadata (VGPR/SGPR counts, spills, LDS) of a HIP shared library
f=${1:?lib}
/opt/rocm/lib/llvm/bin/llvm-objdump --offloading "$f" > /dev/null 2>&1
co="$f.0.hipv4-amdgcn-amd-amdhsa--gfx950"
/opt/rocm/lib/llvm/bin/llvm-readelf --notes "$co" 2>/dev/null | grep -E "^ +\.name:|\.vgpr_count|\.sgpr_count|group_segment_fixed_size|vgpr_spill_count|sgpr_spill_count" | awk '{printf "%s ", $0} /\.vgpr_spill_count/ {print ""}' | sed 's/  */ /g' | cut -c1-260
rm -f "$f".0.*
