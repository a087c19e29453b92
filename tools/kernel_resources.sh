#!/bin/bash
# Per-kernel VGPRs / spills / occupancy of a HIP source for gfx950 (the compiler's
# kernel-resource-usage remarks; device-only compile, nothing written).
#   tools/kernel_resources.sh fhe_amd/csrc/bootstrap.hip [kernel-name-regex] [extra hipcc flags]
src=$1; pat=${2:-.}; shift 2 2>/dev/null
/opt/rocm/bin/hipcc -std=c++17 -O3 --offload-arch=gfx950 --cuda-device-only -c "$src" -o /dev/null \
    -Rpass-analysis=kernel-resource-usage "$@" 2>&1 |
  grep -E "Function Name|remark:     (VGPRs|VGPRs Spill|Occupancy|TotalSGPRs):" |
  sed -E 's/.*Function Name: (\S+).*/\1/; s/.*remark: +([A-Za-z ]+[^:]*): (\S+).*/  \1=\2/' |
  awk -v pat="$pat" '/^_Z/ {show = ($0 ~ pat); if (show) printf "\n%s", $0; next} show {printf " %s", $0} END {print ""}'
