#!/bin/bash
# Per-kernel VGPRs / spills / LDS of an already-built object (fhe_amd/_build/<file>.o) from its code
# object notes, without recompiling:  tools/kres.sh bootstrap [kernel-name-regex]
set -e
o=${1:-bootstrap}; pat=${2:-.}
d=$(mktemp -d)
objcopy -O binary --only-section=.hip_fatbin "$(dirname "$0")/../fhe_amd/_build/$o.o" $d/fat.bin
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 \
    --input=$d/fat.bin --output=$d/k.co
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $d/k.co | awk -v pat="$pat" '
  /\.group_segment_fixed_size:/ {lds=$2} /\.name:/ {name=$2} /\.sgpr_spill_count:/ {ss=$2}
  /\.vgpr_count:/ {v=$2} /\.vgpr_spill_count:/ {vs=$2; if (name ~ pat) printf "%-110s vgpr %s spill %s sspill %s lds %s\n", substr(name,1,110), v, vs, ss, lds}'
rm -rf $d
