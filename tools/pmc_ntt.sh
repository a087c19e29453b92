#!/bin/bash
# Issue / LDS / wait counters of the NTT kernels for A/B builds (abv/<v>.so):
#   tools/pmc_ntt.sh v1 v2 ...   -> gpurun_out/pmc_ntt/<v>/ (one rocprofv3 --pmc pass per variant)
export TMPDIR=/tmp
set -o pipefail
for v in "$@"; do
  FHE_AMD_LIB=abv/$v.so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU \
      SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAVES --kernel-trace --output-format csv \
      -d gpurun_out/pmc_ntt/$v -o run -- python3 tools/ntt_time.py 4096 20 ip 1152921504606830593 > gpurun_out/pmc_ntt_$v.log 2>&1 \
      || { echo "pmc $v failed"; tail -5 gpurun_out/pmc_ntt_$v.log; exit 1; }
  python3 tools/pmc_sum.py gpurun_out/pmc_ntt/$v "$v"
done
