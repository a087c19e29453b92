#!/bin/bash
# round 6: K1x with one gate per workgroup up to one gate per CU -- its tests and the small-batch latency
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r06_k1x_gw}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gates.py tests/test_capi.py tests/test_fb.py -k "std128 or split or k1x or kernel" > gpurun_out/${T}_tests.txt 2>&1 || { tail -c 6000 gpurun_out/${T}_tests.txt; exit 1; }
tail -2 gpurun_out/${T}_tests.txt
timeout -k 10 300 python -u tools/small_batch_time.py 5 > gpurun_out/${T}_latency.txt 2>&1 || { tail -20 gpurun_out/${T}_latency.txt; exit 1; }
cat gpurun_out/${T}_latency.txt
