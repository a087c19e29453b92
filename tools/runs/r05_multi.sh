#!/bin/bash
# Round 5: fused EvalFuncMultiOutput (per-gate test-vector tables), its timing, and the fb / mixed suites after
# the table-buffer change
set -o pipefail
o=gpurun_out/r05_multi_tests.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_fb.py tests/test_mixed.py tests/test_large.py -m gpu > $o 2>&1 || { tail -c 6000 $o; exit 1; }
tail -3 $o
o=gpurun_out/r05_multi_routed.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_backend.py -m gpu -k "routed" > $o 2>&1 || { tail -c 6000 $o; exit 1; }
tail -3 $o
o=gpurun_out/r05_multi_time.txt
timeout -k 10 300 python -u tools/multi_time.py std128 > $o 2>&1 || { cat $o; exit 1; }
cat $o
o=gpurun_out/r05_n2k_tests.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_paramsets.py -m gpu -k "n2k" > $o 2>&1 || { tail -c 6000 $o; exit 1; }
tail -3 $o
