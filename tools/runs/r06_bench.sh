#!/bin/bash
# round-6 check, part 2: the default bench line, rocprofv3 stats of the bench, PMC passes
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r06}
timeout -k 10 500 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo bench-failed; tail -5 gpurun_out/${T}_bench.err; exit 1; }
cat gpurun_out/${T}_bench.json
bash tools/prof_stats.sh ${T}_bench bench.py --no-cpu-baseline || exit 1
bash tools/pmc_run.sh 65536 || exit 1
python3 tools/pmc_traffic.py ${T} 65536 > /dev/null && cp profiles/${T}_pmc_traffic.json gpurun_out/ && echo pmc-summary-ok
