#!/bin/bash
# Round 5: routed mod-Q callers, K1w seam rows vs the reference, K1w q = 2N fallback
set -o pipefail
o=gpurun_out/r05_mixed_backend.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_backend.py -m gpu -k "mod_Q or std256q" > $o 2>&1 || { tail -c 6000 $o; exit 1; }
tail -3 $o
o=gpurun_out/r05_n2k_tests.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_paramsets.py -m gpu -k "n2k" > $o 2>&1 || { tail -c 6000 $o; exit 1; }
tail -3 $o
