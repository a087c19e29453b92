#!/bin/bash
# round-6 check, part 1: the whole GPU suite and smoke() on the shipped library
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r06}
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/${T}_gpu_tests.txt 2>&1 || { tail -c 6000 gpurun_out/${T}_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.txt 2>&1 || { echo smoke-failed; tail -20 gpurun_out/${T}_smoke.txt; exit 1; }
tail -1 gpurun_out/${T}_smoke.txt
