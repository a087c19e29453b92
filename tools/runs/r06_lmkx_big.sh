set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do for k in split wave; do echo -n "$k r$r: "; FHE_HIP_LMK_KERNEL=$k timeout -k 10 300 python -u tools/gate_time.py lmk 4096 16384 65536 2>&1 | grep "^B=" | tr '\n' ' ' || exit 1; echo; done; done
