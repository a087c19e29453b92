#!/bin/bash
# round 6: SQ counters of the small-batch kernels on one gate (K1q, K1x, K1; K1m-4, K1 LMK): where a lone gate's
# waves spend their cycles.  One counter group per pass, each pass under its own kill timeout.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_small
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS"
run() {  # name env method
  local name=$1 envs=$2 m=$3
  env $envs timeout -s KILL 120 rocprofv3 --pmc $G1 --kernel-trace --output-format csv -d gpurun_out/pmc_small/$name -o run \
      -- python3 tools/gate_time.py $m 1 > gpurun_out/pmc_small/$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/pmc_small/$name.log; return 1; }
  python3 tools/pmc_sum.py gpurun_out/pmc_small/$name $name
}
run k1q "FHE_HIP_GINX_KERNEL=qsplit" ginx && run k1x "FHE_HIP_GINX_KERNEL=xsplit" ginx && run k1 "FHE_HIP_GINX_KERNEL=wave" ginx && \
run k1m4 "FHE_HIP_LMK_KERNEL=qsplit" lmk && run k1lmk "FHE_HIP_LMK_KERNEL=wave" lmk
