# round-3 end check of the host-path copy pipeline (since dropped; FHE_HIP_HOST_PIPELINE=0 was its
# A/B knob and is a no-op now): seam timings, every GPU test, smoke()
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/seam_time.py ginx 1 16 256 1024 8192 16384 65536 > gpurun_out/r03_seam_ginx_final.txt 2>&1 || { echo seam-failed; tail -5 gpurun_out/r03_seam_ginx_final.txt; exit 1; }
timeout -k 10 200 python -u tools/seam_time.py lmk 1 1024 8192 65536 > gpurun_out/r03_seam_lmk_final.txt 2>&1 || { echo seam-lmk-failed; exit 1; }
FHE_HIP_HOST_PIPELINE=0 timeout -k 10 200 python -u tools/seam_time.py ginx 16384 65536 > gpurun_out/r03_seam_ginx_oneshot.txt 2>&1 || { echo seam-oneshot-failed; exit 1; }
grep -h B= gpurun_out/r03_seam_ginx_final.txt gpurun_out/r03_seam_ginx_oneshot.txt gpurun_out/r03_seam_lmk_final.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r03_gputest_end2.txt 2>&1 || { echo pytest-failed; tail -30 gpurun_out/r03_gputest_end2.txt; exit 1; }
tail -1 gpurun_out/r03_gputest_end2.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03_smoke_end2.txt 2>&1 || { echo smoke-failed; tail -20 gpurun_out/r03_smoke_end2.txt; exit 1; }
tail -1 gpurun_out/r03_smoke_end2.txt
echo end-done
