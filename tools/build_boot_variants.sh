#!/bin/bash
# A/B variants that differ only in one HIP file's macros (SRC, default bootstrap): that file recompiled with
# the flags, linked with the other objects of the current build (fhe_amd/_build, make first) into
# abv/<name>.so.  The variants build in parallel.
#   [SRC=ntt] tools/build_boot_variants.sh name1 "-DFOO=1" name2 "-DBAR=2" ...
set -e
cd "$(dirname "$0")/.."
src=${SRC:-bootstrap}
mkdir -p abv
names=()
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  mkdir -p abv/obj_$name
  (/opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics $flags \
     -c fhe_amd/csrc/$src.hip -o abv/obj_$name/$src.o &&
   /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o abv/$name.so abv/obj_$name/$src.o \
     $(ls fhe_amd/_build/*.o | grep -v "/$src.o\$") -lgomp && echo "built abv/$name.so ($flags)") &
done
wait
