#!/bin/bash
# prime-qKS key switch (TOY, SIGNED_MOD_TEST) on the u32-row tiled kernel: parity vs the reference's KeySwitch and
# the gate goldens, then gate throughput against the u64 row gathers (FHE_HIP_KS32=0), two rounds
set -e
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_paramsets.py tests/test_large.py tests/test_backend.py tests/test_capi.py tests/test_mixed.py tests/test_fb.py -m gpu -k "toy or signed_mod" > gpurun_out/r06_ksprime_tests.txt 2>&1 || { tail -c 5000 gpurun_out/r06_ksprime_tests.txt; exit 1; }
tail -2 gpurun_out/r06_ksprime_tests.txt
for round in 1 2; do
  for ks in 1 0; do
    echo "KS32=$ks r$round:"; FHE_HIP_KS32=$ks timeout -k 10 300 python tools/bench_sets.py toy signed_mod_test toy_lmkcdey 2>&1 | grep -v "^keygen\|^load"
  done
done
