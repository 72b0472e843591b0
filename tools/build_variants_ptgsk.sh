#!/bin/bash
# Fast variant build: recompile only kernels/ptgsk.hip with extra flags and link it with the
# regular objects in shyft_amd/csrc/_obj (run `make -C shyft_amd/csrc` first).
# usage: build_variants_ptgsk.sh name1 "flags1" name2 "flags2" ...
set -e
cd "$(dirname "$0")/../shyft_amd/csrc"
OUTD=${OUT:-tools/variants}; mkdir -p ../../$OUTD
others=$(ls _obj/*.o _obj/kernels/*.o | grep -v "kernels/ptgsk.o")
while [ $# -gt 1 ]; do
  name=$1; flags=$2; shift 2
  (/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off $flags -c kernels/ptgsk.hip -o /tmp/ptgsk_$name.o &&
   /opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared -o ../../$OUTD/$name.so $others /tmp/ptgsk_$name.o -lrocblas -lrccl &&
   echo built $name) &
done
wait
