#!/bin/bash
# Round 4: the C-API GPU test on its own (a hang dumps every thread's stack at 120 s), then the rest of the
# new GPU tests.
set -o pipefail
export FHE_SEGV_TRACE=1
timeout -k 10 170 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_backend.py -m gpu -k "c_api" > gpurun_out/r04_capi.txt 2>&1 || { tail -c 8000 gpurun_out/r04_capi.txt; exit 1; }
tail -3 gpurun_out/r04_capi.txt
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_backend.py tests/test_ntt.py tests/test_cereal.py -m gpu -k "(refresh or ntt4096 or context or std128_3 or std128_4_lmkcdey) and not c_api" > gpurun_out/r04_routed2.txt 2>&1 || { tail -c 6000 gpurun_out/r04_routed2.txt; exit 1; }
tail -3 gpurun_out/r04_routed2.txt
