#!/bin/bash
# Kernel resource usage (VGPRs, SGPRs, spills, LDS) of the gfx950 code object inside a built
# object file: tools/kres.sh [build/rt_kernels.o] [name-regex]
set -e
OBJ=${1:-raytracing-tests_amd/build/rt_kernels.o}
PAT=${2:-inw_pm|inw_sm}
LLVM=/opt/rocm/lib/llvm/bin
T=$(mktemp -d)
$LLVM/llvm-objcopy --dump-section=.hip_fatbin=$T/fat.bin "$OBJ"
$LLVM/clang-offload-bundler --unbundle --type=o --input=$T/fat.bin \
    --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/k.co
$LLVM/llvm-readelf --notes $T/k.co | grep -E "^ +\.(name|vgpr_count|sgpr_count|vgpr_spill_count|sgpr_spill_count|group_segment_fixed_size):" |
    awk '/\.group_segment_fixed_size:/{lds=$2} /\.name:/{name=$2} /\.sgpr_count:/{s=$2} /\.sgpr_spill_count:/{ss=$2}
         /\.vgpr_count:/{v=$2} /\.vgpr_spill_count:/{vs=$2; printf "%-70s vgpr %4s spill %3s sgpr %3s spill %3s lds %6s\n", name, v, vs, s, ss, lds}' |
    grep -E "$PAT" || true
rm -rf $T
