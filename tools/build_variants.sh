#!/bin/bash
# Variant build of one kernel file: recompile kernels/<kernel>.hip with extra flags and link it with the
# regular objects in shyft_amd/csrc/_obj (run `make -C shyft_amd/csrc` first). Output: <outdir>/<name>.so,
# loaded by setting SHYFT_HIP_LIB.
# usage: build_variants.sh <kernel> <outdir> name1 "flags1" name2 "flags2" ...
set -e
kernel=$1; out=$(realpath -m "$2"); shift 2
cd "$(dirname "$0")/../shyft_amd/csrc"
mkdir -p "$out"
others=$(ls _obj/*.o _obj/kernels/*.o | grep -v "kernels/$kernel.o")
while [ $# -gt 1 ]; do
  name=$1; flags=$2; shift 2
  (/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off $flags -c kernels/$kernel.hip -o /tmp/${kernel}_$name.o &&
   /opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared -o "$out/$name.so" $others /tmp/${kernel}_$name.o -lrocblas -lrccl &&
   echo built $name) &
done
wait
