# round-3 final check, part A: every GPU test (timed: the driver allows 900 s), smoke(), the 2-rank rehearsal
set -o pipefail
mkdir -p gpurun_out
start=$(date +%s)
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r03_gputest_all.txt 2>&1 || { echo pytest-failed; tail -30 gpurun_out/r03_gputest_all.txt; exit 1; }
echo "pytest wall $(( $(date +%s) - start )) s"
tail -2 gpurun_out/r03_gputest_all.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03_smoke.txt 2>&1 || { echo smoke-failed; tail -20 gpurun_out/r03_smoke.txt; exit 1; }
tail -1 gpurun_out/r03_smoke.txt
echo part-a-done
