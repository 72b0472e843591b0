#!/bin/bash
# Variant libraries of one kernel source: recompile shyft_amd/csrc/kernels/<kernel>.hip with extra flags and link it
# with the regular objects of the tree (run `make -C shyft_amd/csrc` first).
# usage: build_variant_kernel.sh <kernel> name1 "flags1" [name2 "flags2" ...]   -> tools/vlib/<name>.so
set -e
cd "$(dirname "$0")/../shyft_amd/csrc"
k=$1; shift
mkdir -p ../../tools/vlib
others=$(ls _obj/*.o _obj/kernels/*.o | grep -v "kernels/$k.o")
while [ $# -gt 1 ]; do
  name=$1; flags=$2; shift 2
  (/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off $flags -c kernels/$k.hip -o /tmp/v_${k}_$name.o 2>/dev/null &&
   /opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared -o ../../tools/vlib/$name.so $others /tmp/v_${k}_$name.o -lrocblas -lrccl &&
   echo built $name) &
done
wait
