#!/bin/bash
# Round 5: tiled key switch at baseKS 21 (STD256Q_3), key fan-out test, 60-bit NTT pair-ordered loads (A/B)
set -o pipefail
o=gpurun_out/r05_ks21_tests.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_paramsets.py tests/test_capi.py -m gpu -k "keyswitch or std256q_3 or copy_keys or seam" > $o 2>&1 || { tail -c 6000 $o; exit 1; }
tail -3 $o
o=gpurun_out/r05_ks21_bench.txt; : > $o
for r in 1 2; do
  for ks in 1 0; do
    echo "== FHE_HIP_KS32=$ks r$r" >> $o
    FHE_HIP_KS32=$ks timeout -k 10 300 python -u tools/bench_sets.py std256q_3 >> $o 2>&1 || { cat $o; exit 1; }
  done
done
cat $o
cp fhe_amd/libfhe_amd.so abv/base.so
o=gpurun_out/r05_ntt64_pairload.txt
timeout -k 10 300 bash tools/ntt64_ab.sh base ntt64pl > $o 2>&1 || { cat $o; exit 1; }
cat $o
# config 3: K1 vs the split kernel K1s (two waves per gate) at 2 and 1 gates per workgroup
o=gpurun_out/r05_split1024.txt; : > $o
for r in 1 2; do
  for v in "base " "base split" "g2one split"; do
    set -- $v
    echo -n "$1 ${2:-k1} r$r: " >> $o
    FHE_AMD_LIB=abv/$1.so FHE_HIP_GINX_KERNEL=${2:-auto} timeout -k 10 120 python tools/gate_time.py ginx 1024 4096 2>&1 | grep "B=" | tr '\n' ' ' >> $o || { cat $o; exit 1; }
    echo >> $o
  done
done
cat $o
# config 3's stall profile: the two SQ passes of pmc_run.sh at 1024 gates (one wave per SIMD)
export TMPDIR=/tmp
for i in 1 2; do
  grp="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
  [ $i = 2 ] && grp="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM"
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmc1024/p$i -o run -- python3 tools/pmc_workload.py 1024 nontt > /dev/null 2>&1 || { echo pmc-failed; exit 1; }
done
echo pmc1024-done
