#!/bin/bash
# Do co-resident waves that start together stay in lockstep?  K1 at 2048 gates (one round of two waves per
# SIMD) and K1x at 1024 with the odd workgroup slot of each CU at priority 1 (prio) or started late (stag)
set -e
for round in 1 2; do
  for v in base k1prio k1stag; do
    lib=fhe_amd/libfhe_amd.so; [ $v != base ] && lib=abv/$v.so
    echo -n "K1 $v r$round: "; FHE_HIP_GINX_KERNEL=wave FHE_AMD_LIB=$lib timeout -k 10 120 python tools/gate_time.py ginx 1024 2048 4096 2>&1 | grep "B=" | sed 's/ms.batch.*correct=/ms /' | tr '\n' ' '; echo
  done
  for v in base xprio2 xstag2; do
    lib=fhe_amd/libfhe_amd.so; [ $v != base ] && lib=abv/$v.so
    echo -n "K1x $v r$round: "; FHE_HIP_GINX_KERNEL=xsplit FHE_AMD_LIB=$lib timeout -k 10 120 python tools/gate_time.py ginx 512 1024 2>&1 | grep "B=" | sed 's/ms.batch.*correct=/ms /' | tr '\n' ' '; echo
  done
done
