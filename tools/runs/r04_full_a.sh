#!/bin/bash
# Round 4: the whole GPU suite (after the K1w LMKCDEY form, the 32-bit key switch on the 64-bit path and the
# context-owned seam scratch)
set -o pipefail
export FHE_SEGV_TRACE=1
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r04_gpu_tests_b.txt 2>&1; rc=$?
grep -E "FAILED|passed|failed|error" gpurun_out/r04_gpu_tests_b.txt | tail -5
exit $rc
