#!/bin/bash
# Round 4: K1w (N = 2048 GINX in registers) parity and rate on STD256Q, then the crash isolation of the
# routed-gate test.
set -o pipefail
timeout -k 10 400 python -u -X faulthandler -m pytest -x -v --timeout 300 --timeout-method thread tests/test_paramsets.py -m gpu -k "n2k or std256q" 2>&1 | tee gpurun_out/r04_n2k_tests.txt || exit 1
for flag in 1 0; do
  echo "FHE_HIP_N2K=$flag"; FHE_HIP_N2K=$flag timeout -k 10 200 python -u tools/bench_sets.py std256q 2>&1 | tee -a gpurun_out/r04_n2k_bench.txt || exit 1
done
timeout -k 10 300 python -u -X faulthandler -m pytest -x -v --timeout 200 --timeout-method thread tests/test_backend.py -m gpu -k "routed_gate and lmkcdey" 2>&1 | tee gpurun_out/r04_dbg1.txt || exit 1
timeout -k 10 300 python -u -X faulthandler -m pytest -x -v --timeout 200 --timeout-method thread tests/test_backend.py -m gpu -k "routed_gate" 2>&1 | tee gpurun_out/r04_dbg2.txt
