#!/bin/bash
# 60-bit NTT (k_ntt1024w64, 4096 polynomials, 4 waves per SIMD) where the non-VALU cycles go: SQ issue / wait
# counters, VMEM and LDS in-flight levels (Little's law latency), then the two-rank bench rehearsal on one GPU
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out/pmc_ntt6
Q=1152921504606830593
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc_ntt6 -o p1 -- python3 tools/ntt_time.py 4096 20 ip $Q
timeout -s KILL 120 rocprofv3 --pmc SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR --kernel-trace --output-format csv -d gpurun_out/pmc_ntt6 -o p2 -- python3 tools/ntt_time.py 4096 20 ip $Q
FHE_BENCH_DEVICE_MAP=0,0 FHE_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/r06_bench_rehearsal_w2.json 2> gpurun_out/r06_bench_rehearsal_w2.err
echo done
