# round 3, GPU call A: the seam for every parameter set, config-3 parity, the 2-rank rehearsal
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_backend.py tests/test_full.py -k "backend or config3" -m gpu -x -v \
    --timeout 400 --timeout-method thread > gpurun_out/r03_a_tests.log 2>&1 || { echo tests-failed; tail -40 gpurun_out/r03_a_tests.log; exit 1; }
tail -3 gpurun_out/r03_a_tests.log
FHE_BENCH_DEVICE_MAP=0,0 FHE_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 3 --warmup 1 \
    --no-cpu-baseline > gpurun_out/r03_bench_rehearsal_w2.json 2> gpurun_out/r03_bench_rehearsal_w2.err || { echo rehearsal-failed; tail -20 gpurun_out/r03_bench_rehearsal_w2.err; exit 1; }
cat gpurun_out/r03_bench_rehearsal_w2.json
echo all-done
