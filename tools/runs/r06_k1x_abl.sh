#!/bin/bash
# K1x timing-only ablations (wrong results by design): no barrier (xabl1), no key loads (xabl2) vs default
set -e
for round in 1 2; do
  for v in base xabl1 xabl2; do
    lib=fhe_amd/libfhe_amd.so; [ $v != base ] && lib=abv/$v.so
    echo -n "$v r$round: "; FHE_HIP_GINX_KERNEL=xsplit FHE_AMD_LIB=$lib timeout -k 10 120 python tools/gate_time.py ginx 512 1024 2>&1 | grep "B=" | sed 's/ms.batch.*correct=/ms /' | tr '\n' ' '; echo
  done
done
