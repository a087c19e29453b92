#!/bin/bash
# round 6: K1m's two-digit form as LMKCDEY's small-batch kernel -- its parity test, the LMKCDEY goldens that now
# run on it by default, and the small-batch latency against K1 LMK
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r06_lmkx}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gates.py -k "lmk or lmkcdey" > gpurun_out/${T}_tests1.txt 2>&1 || { tail -c 6000 gpurun_out/${T}_tests1.txt; exit 1; }
tail -2 gpurun_out/${T}_tests1.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_fb.py tests/test_multi_gates.py tests/test_mixed.py tests/test_backend.py tests/test_paramsets.py -k "lmk or LMK or medium or MEDIUM" \
    > gpurun_out/${T}_tests2.txt 2>&1 || { tail -c 6000 gpurun_out/${T}_tests2.txt; exit 1; }
tail -2 gpurun_out/${T}_tests2.txt
timeout -k 10 300 python -u tools/small_batch_time.py 5 STD128_LMKCDEY LMKCDEY > gpurun_out/${T}_latency.txt 2>&1 || { tail -20 gpurun_out/${T}_latency.txt; exit 1; }
cat gpurun_out/${T}_latency.txt
