#!/bin/bash
# Round 5: the 2-rank bench path on the box's one GPU (gloo barrier/max, both ranks on device 0)
set -o pipefail
FHE_BENCH_DEVICE_MAP=0,0 FHE_BENCH_BACKEND=gloo timeout -k 10 900 python bench.py --gpus 2 --no-cpu-baseline > gpurun_out/r05_bench_rehearsal_w2_one_gpu.json 2> gpurun_out/r05_bench_rehearsal.err || { tail -20 gpurun_out/r05_bench_rehearsal.err; exit 1; }
cat gpurun_out/r05_bench_rehearsal_w2_one_gpu.json
