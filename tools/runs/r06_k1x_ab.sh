#!/bin/bash
# K1x (k_blind_rotate_ginx2x) A/B at 512 / 1024 gates: variants from tools/build_boot_variants.sh, two
# interleaved rounds; then PMC (SQ issue / wait counters) of the default K1x and of K1 at 1024 gates
export TMPDIR=/tmp
set -e
for round in 1 2; do
  for v in base xk4t2 xprio xstag; do
    lib=fhe_amd/libfhe_amd.so; [ $v != base ] && lib=abv/$v.so
    echo -n "$v r$round: "; FHE_AMD_LIB=$lib timeout -k 10 120 python tools/gate_time.py ginx 512 1024 2>&1 | grep "B=" | tr '\n' ' '; echo
  done
done
mkdir -p gpurun_out/pmc_k1x
for k in xsplit wave; do
  FHE_HIP_GINX_KERNEL=$k timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU --kernel-trace --output-format csv -d gpurun_out/pmc_k1x/$k -o p1 -- python3 tools/gate_time.py ginx 1024
  FHE_HIP_GINX_KERNEL=$k timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM --kernel-trace --output-format csv -d gpurun_out/pmc_k1x/$k -o p2 -- python3 tools/gate_time.py ginx 1024
done
echo done
