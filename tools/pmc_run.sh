#!/bin/bash
# rocprofv3 PMC passes (counters only with --kernel-trace; one counter group per pass),
# run from the repo root: the workload (tools/pmc_workload.py <B>) and the FETCH/WRITE
# calibration binary (build/calib_fetch).  Outputs under gpurun_out/pmc/.
export TMPDIR=/tmp
set -e
B=${1:-65536}
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmc/p$i -o run -- python3 tools/pmc_workload.py $B
done
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc/c3 -o run -- build/calib_fetch
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc/c4 -o run -- build/calib_fetch
echo pmc done
