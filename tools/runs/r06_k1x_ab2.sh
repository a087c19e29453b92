#!/bin/bash
# K1x with the exchange buffer as the forward NTT's second tile (default) vs one tile (xt1) and 4-gate
# workgroups (xk4); parity of the default first
set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread "tests/test_gates.py::test_gpu_split_ginx_kernel_bit_exact[xsplit]" tests/test_full.py::test_gpu_config3_batch_bit_exact
for round in 1 2; do
  for v in base xt1 xk4 wave; do
    lib=fhe_amd/libfhe_amd.so; [ $v != base ] && [ $v != wave ] && lib=abv/$v.so
    k=xsplit; [ $v = wave ] && k=wave
    echo -n "$v r$round: "; FHE_HIP_GINX_KERNEL=$k FHE_AMD_LIB=$lib timeout -k 10 120 python tools/gate_time.py ginx 256 512 768 1024 2>&1 | grep "B=" | sed 's/ms.batch.*correct=/ms /' | tr '\n' ' '; echo
  done
done
