#!/bin/bash
# LDS / issue counters of the blind-rotation kernels for A/B ablation builds (abv/<v>.so):
#   tools/pmc_lds.sh <B> v1 v2 ...   -> gpurun_out/pmc_lds/<v>/ (one rocprofv3 --pmc pass per variant)
export TMPDIR=/tmp
set -o pipefail
B=$1; shift
for v in "$@"; do
  FHE_AMD_LIB=abv/$v.so timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
      SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_INSTS_VALU --kernel-trace --output-format csv \
      -d gpurun_out/pmc_lds/$v -o run -- python3 tools/pmc_workload.py $B nontt > gpurun_out/pmc_lds_$v.log 2>&1 \
      || { echo "pmc $v failed"; tail -5 gpurun_out/pmc_lds_$v.log; exit 1; }
  python3 tools/pmc_sum.py gpurun_out/pmc_lds/$v "$v"
done
