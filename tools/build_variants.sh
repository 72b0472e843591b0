#!/bin/bash
# Build libshyft_hip.so variants with different kernel compile flags into tools/variants/<name>.so
# usage: build_variants.sh name1 "flags1" name2 "flags2" ...
set -e
cd "$(dirname "$0")/../shyft_amd/csrc"
mkdir -p ../../tools/variants
while [ $# -gt 1 ]; do
  name=$1; flags=$2; shift 2
  rm -rf _vobj_$name; mkdir -p _vobj_$name/kernels
  for f in $(grep "^SRCS :=" Makefile | cut -d= -f2); do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off $flags -c $f -o _vobj_$name/${f%.hip}.o &
  done
  wait
  /opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared -o ../../tools/variants/$name.so _vobj_$name/*.o _vobj_$name/kernels/*.o
  rm -rf _vobj_$name
  echo built $name
done
