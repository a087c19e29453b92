#!/bin/bash
# Round 4: K1w-LMKCDEY at 2^28 <= Q < 2^29 (STD256_3 / STD256_4_LMKCDEY): parity against the 64-bit / A32
# accumulator and the reference goldens, then the rate with and without it.
set -o pipefail
export FHE_SEGV_TRACE=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_paramsets.py -m gpu -k "n2k or lmkcdey" > gpurun_out/r04_qm2_tests.txt 2>&1 || { tail -c 6000 gpurun_out/r04_qm2_tests.txt; exit 1; }
tail -3 gpurun_out/r04_qm2_tests.txt
for flag in 1; do
  echo "FHE_HIP_N2K=$flag" >> gpurun_out/r04_qm2_bench.txt; FHE_HIP_N2K=$flag timeout -k 10 200 python -u tools/bench_sets.py std256q_4_lmkcdey std256_3_lmkcdey std256_4_lmkcdey std256q_lmkcdey std256q_3_lmkcdey std256q >> gpurun_out/r04_qm2_bench.txt 2>&1 || exit 1
done
cat gpurun_out/r04_qm2_bench.txt
