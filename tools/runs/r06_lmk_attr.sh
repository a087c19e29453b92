#!/bin/bash
# (1) K1x parity after the monomial prefetch; (2) K1x A/B; (3) LMKCDEY op-list kernel attribution: timing-only
# ablations (FHE_LMK_ABL bits: 1 EXT keys cache-resident, 2 AUTO keys cache-resident, 4 automorphism gathers
# linear, 8 no EXT digit exchange); (4) PMC of k_blind_rotate_lmk at 16,384 gates
export TMPDIR=/tmp
set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread "tests/test_gates.py::test_gpu_split_ginx_kernel_bit_exact[xsplit]" tests/test_full.py::test_gpu_config3_batch_bit_exact tests/test_capi.py::test_gpu_gate_kernel_reports_the_launched_kernel
for round in 1 2; do
  for v in base xmpf0 xk4; do
    echo -n "K1x $v r$round: "; FHE_HIP_GINX_KERNEL=xsplit FHE_AMD_LIB=abv/$v.so timeout -k 10 120 python tools/gate_time.py ginx 512 1024 2>&1 | grep "B=" | sed 's/ms.batch.*correct=/ms /' | tr '\n' ' '; echo
  done
done
for round in 1 2; do
  for v in base lab1 lab2 lab4 lab8; do
    echo -n "LMK $v r$round: "; FHE_AMD_LIB=abv/$v.so timeout -k 10 120 python tools/gate_time.py lmk 16384 2>&1 | grep "B=" | sed 's/ms.batch.*correct=/ms /' | tr '\n' ' '; echo
  done
done
timeout -k 10 60 rocprofv3 --list-avail > gpurun_out/r06_avail.txt 2>&1 || true
mkdir -p gpurun_out/pmc_lmk
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS --kernel-trace --output-format csv -d gpurun_out/pmc_lmk -o p1 -- python3 tools/gate_time.py lmk 16384
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc_lmk -o p2 -- python3 tools/gate_time.py lmk 16384
echo done
