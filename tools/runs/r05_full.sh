#!/bin/bash
# round-5 check: the whole GPU suite, smoke(), the default bench line, rocprofv3 stats of the bench, PMC passes
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/${T}_gpu_tests.txt 2>&1 || { tail -c 6000 gpurun_out/${T}_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.txt 2>&1 || { echo smoke-failed; tail -20 gpurun_out/${T}_smoke.txt; exit 1; }
tail -1 gpurun_out/${T}_smoke.txt
timeout -k 10 500 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo bench-failed; tail -5 gpurun_out/${T}_bench.err; exit 1; }
cat gpurun_out/${T}_bench.json
bash tools/prof_stats.sh ${T}_bench bench.py --no-cpu-baseline || exit 1
bash tools/pmc_run.sh 65536 || exit 1
python3 tools/pmc_traffic.py ${T} 65536 > /dev/null && cp profiles/${T}_pmc_traffic.json gpurun_out/ && echo pmc-summary-ok
