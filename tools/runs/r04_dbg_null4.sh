#!/bin/bash
# Round 4: the std192_lmkcdey null-accumulator failure with engine diagnostics
set -o pipefail
export FHE_HIP_DEBUG=1
timeout -k 10 300 python -u -m pytest -v -s --timeout 200 --timeout-method thread tests/test_backend.py -m gpu -k "std192_lmkcdey" > gpurun_out/r04_n4.txt 2>&1; rc=$?
grep -E "PASSED|FAILED|fhe_hip\]" gpurun_out/r04_n4.txt | head -40
[ $rc -gt 1 ] && exit $rc
exit 0
