#!/bin/bash
# IDW gather variants: kernels/idw.hip with tools/patches/idw_row_groups.patch applied (G-row temperature groups,
# occupancy target, height difference from LDS), compiled with the knobs given and linked with the regular objects.
# usage: build_variants_idw.sh name1 "flags1" ...   -> tools/vlib/<name>.so   (run `make -C shyft_amd/csrc` first)
set -e
cd "$(dirname "$0")/../shyft_amd/csrc"
mkdir -p ../../tools/vlib
cp kernels/idw.hip /tmp/idw_rg.hip
patch -s /tmp/idw_rg.hip < ../../tools/patches/idw_row_groups.patch
cp /tmp/idw_rg.hip kernels/_idw_rg.hip
others=$(ls _obj/*.o _obj/kernels/*.o | grep -v "kernels/idw.o")
while [ $# -gt 1 ]; do
  name=$1; flags=$2; shift 2
  (/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off $flags -c kernels/_idw_rg.hip -o /tmp/idw_$name.o 2>/dev/null &&
   /opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared -o ../../tools/vlib/$name.so $others /tmp/idw_$name.o -lrocblas -lrccl &&
   echo built $name) &
done
wait
rm -f kernels/_idw_rg.hip
