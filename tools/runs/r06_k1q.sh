#!/bin/bash
# round 6: K1q (four waves per gate) -- its tests, the GINX goldens that run on it by default, and the latency
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r06_k1q}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gates.py tests/test_capi.py tests/test_fb.py tests/test_multi_gates.py tests/test_backend.py \
    -k "std128 or split or k1x or kernel" > gpurun_out/${T}_tests.txt 2>&1 || { tail -c 6000 gpurun_out/${T}_tests.txt; exit 1; }
tail -2 gpurun_out/${T}_tests.txt
timeout -k 10 300 python -u tools/small_batch_time.py 5 > gpurun_out/${T}_latency.txt 2>&1 || { tail -20 gpurun_out/${T}_latency.txt; exit 1; }
cat gpurun_out/${T}_latency.txt
timeout -k 10 200 python -u tools/gate_time.py ginx 1 64 256 257 512 > gpurun_out/${T}_gate_time.txt 2>&1 || { tail -20 gpurun_out/${T}_gate_time.txt; exit 1; }
grep "^B=" gpurun_out/${T}_gate_time.txt
