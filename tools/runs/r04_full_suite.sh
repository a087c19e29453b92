#!/bin/bash
# round 4: the whole GPU suite with the current defaults, then smoke() and the default bench line
set -o pipefail
mkdir -p gpurun_out
export FHE_SEGV_TRACE=1
timeout -k 10 1000 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/r04_gpu_suite.txt 2>&1 || { tail -c 6000 gpurun_out/r04_gpu_suite.txt; exit 1; }
tail -3 gpurun_out/r04_gpu_suite.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04_smoke2.txt 2>&1 || { echo smoke-failed; tail -20 gpurun_out/r04_smoke2.txt; exit 1; }
tail -1 gpurun_out/r04_smoke2.txt
timeout -k 10 500 python bench.py > gpurun_out/r04_bench2.json 2> gpurun_out/r04_bench2.err || { echo bench-failed; tail -5 gpurun_out/r04_bench2.err; exit 1; }
cat gpurun_out/r04_bench2.json
