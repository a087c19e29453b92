#!/bin/bash
# Round 4: SQ counters of K1w (k_blind_rotate_n2k) on STD256Q (tools/bench_sets.py, B = 2048), two passes.
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out/pmc_n2k
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmc_n2k/p$i -o run -- python3 tools/bench_sets.py std256q
done
python3 tools/pmc_sum.py gpurun_out/pmc_n2k n2k > gpurun_out/pmc_n2k/summary.txt
cat gpurun_out/pmc_n2k/summary.txt
