set -o pipefail
for v in w4r1 w3r1; do
  FHE_AMD_LIB=abv/$v.so timeout -k 10 200 python -u -m pytest tests/test_large.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/wab_test_$v.log 2>&1 || { echo "$v tests failed"; tail -5 gpurun_out/wab_test_$v.log; exit 1; }
  echo "$v tests ok"
done
for round in 1 2; do
for v in w3r0 w4r0 w3r1 w4r1; do
  echo -n "$v: "; FHE_AMD_LIB=abv/$v.so timeout -k 10 120 python tools/bench_large.py --batch 2048 --steps 2 --sign-batch 64 || exit 1
done
done
