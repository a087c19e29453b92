# round-2 final check, part A: every GPU test, smoke(), the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_gputest_all.txt 2>&1 || { echo pytest-failed; tail -20 gpurun_out/r02_gputest_all.txt; exit 1; }
tail -2 gpurun_out/r02_gputest_all.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r02_smoke.txt 2>&1 || { echo smoke-failed; tail -20 gpurun_out/r02_smoke.txt; exit 1; }
tail -1 gpurun_out/r02_smoke.txt
timeout -k 10 400 python bench.py > gpurun_out/r02_bench.json 2> gpurun_out/r02_bench.err || { echo bench-failed; tail -5 gpurun_out/r02_bench.err; exit 1; }
echo part-a-done
