#!/bin/bash
# Round 4: K1w-LMKCDEY with 4 digits (parity), the u32 key-switch check, then the final-B evidence run
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_paramsets.py -m gpu -k "n2k or std256q_4_lmkcdey or std256q_lmkcdey" > gpurun_out/r04_nd4_tests.txt 2>&1 || { tail -c 5000 gpurun_out/r04_nd4_tests.txt; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r04_nd4_tests.txt | tail -6
bash tools/runs/r04_ksw.sh || exit $?
bash tools/runs/r04_final_b.sh
