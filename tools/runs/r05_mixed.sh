#!/bin/bash
# Round 5: mod-Q inputs (SwitchCTtoqn prelude), seam repeat, K1w q = 2N fallback, routed mixed callers
set -o pipefail
o=gpurun_out/r05_mixed_tests.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_mixed.py tests/test_capi.py -m gpu > $o 2>&1 || { tail -c 6000 $o; exit 1; }
tail -3 $o
o=gpurun_out/r05_mixed_backend.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_backend.py -m gpu -k "mod_Q or std256q" > $o 2>&1 || { tail -c 6000 $o; exit 1; }
tail -3 $o
o=gpurun_out/r05_n2k_tests.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_paramsets.py -m gpu -k "n2k" > $o 2>&1 || { tail -c 6000 $o; exit 1; }
tail -3 $o
