#!/bin/bash
# icache counters for each variant: tools/pmc_icache.sh variant...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  FHE_AMD_LIB=build/variants/$v.so timeout -k 10 300 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES --kernel-trace --output-format csv -d gpurun_out/icache/$v -o run -- python3 tools/gate_time.py ginx 8192 > /dev/null 2>&1 || exit 1
done
