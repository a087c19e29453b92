#!/bin/bash
# Build A/B variants of libfhe_amd.so into abv/<name>.so.
#   tools/build_variants.sh name1 "-DFOO=1" name2 "-DBAR=2" ...
set -e
cd "$(dirname "$0")/.."
mkdir -p abv
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  out=abv/obj_$name; mkdir -p $out
  for f in fhe_amd/csrc/*.hip; do
    /opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC --offload-arch=gfx950 $flags -c $f -o $out/$(basename $f .hip).o &
  done
  for f in fhe_amd/csrc/*.cpp; do
    g++ -std=c++17 -O3 -fPIC -fopenmp -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ $flags -c $f -o $out/$(basename $f .cpp).o &
  done
  wait
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o abv/$name.so $out/*.o -lgomp
  echo "built abv/$name.so ($flags)"
done
