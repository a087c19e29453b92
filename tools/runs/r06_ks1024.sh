#!/bin/bash
# K2 with 1024-gate tiles (one thread per gate, 1024-thread workgroups) vs the 512-gate tiles at 32,768 and
# 65,536 gates: time (two rounds) and the PMC traffic of one launch set
export TMPDIR=/tmp
set -e
for round in 1 2; do
  for v in base ks1024; do
    echo -n "$v r$round: "; FHE_AMD_LIB=abv/$v.so timeout -k 10 200 python tools/ks_time.py 65536 20 2>&1 | tail -1
    echo -n "$v r$round 32768: "; FHE_AMD_LIB=abv/$v.so timeout -k 10 200 python tools/ks_time.py 32768 20 2>&1 | tail -1
  done
done
for v in base ks1024; do
  FHE_AMD_LIB=abv/$v.so timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_ks/$v -o f -- python3 tools/ks_time.py 65536 3
  FHE_AMD_LIB=abv/$v.so timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_ks/$v -o w -- python3 tools/ks_time.py 65536 3
done
echo done
