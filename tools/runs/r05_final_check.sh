#!/bin/bash
# Round 5 close: smoke() and the gate / full-path GPU tests on the shipped library (rebuilt from the committed source)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05_final_smoke.txt 2>&1 || { tail -20 gpurun_out/r05_final_smoke.txt; exit 1; }
tail -1 gpurun_out/r05_final_smoke.txt
o=gpurun_out/r05_final_gpu_tests.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gates.py tests/test_full.py tests/test_mixed.py -m gpu > $o 2>&1 || { tail -c 6000 $o; exit 1; }
tail -2 $o
