#!/bin/bash
# Regenerates every key-dependent golden fixture from the reference (oracle/_ref), one process per
# group (the reference's memory stays bounded).  Usage: tools/regen_goldens.sh [groups...]
# groups: gates wider multi fb large config3 full  (default: all of them)
set -e
cd "$(dirname "$0")/.."
G=tests/golden/make_golden.py
# private copies of the libraries: rebuilding the tree's libraries under a running generator would
# replace the mapped files
L=$(mktemp -d /tmp/regen_libs.XXXX)
cp fhe_amd/libfhe_amd.so oracle/_ref/libfhe_ref.so "$L"/
export FHE_AMD_LIB="$L/libfhe_amd.so" FHE_REF_SO="$L/libfhe_ref.so"
groups=${@:-gates wider multi fb large config3 full}
for g in $groups; do
  case $g in
    gates)  for s in std128 lmkcdey ap; do python $G gates $s; done ;;
    wider)  for s in $(python -c "import sys; sys.path.insert(0,'tests/golden'); sys.path.insert(0,'tests'); from make_golden import WIDER_SETS; print(' '.join(WIDER_SETS))"); do python $G wider $s; done ;;
    multi)  python $G multi std128; python $G multi lmkcdey ;;
    fb)     python $G fb std128; python $G fb lmkcdey ;;
    large)  for s in $(python -c "import sys; sys.path.insert(0,'tests/golden'); sys.path.insert(0,'tests'); from make_golden import LARGE_SETS; print(' '.join(LARGE_SETS))"); do python $G large $s; done ;;
    config3) python $G config3 ;;
    full)   python $G full std128; python $G full lmkcdey ;;
    fulllmk) python $G full lmkcdey ;;
  esac
  echo "== $g done $(date +%T)"
done
