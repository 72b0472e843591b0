#!/bin/bash
# Test-only racy variant of the pt_gs_k kernel (round 4's 750ee49 aliasing): the Brent results are written over the
# jobs' z1 slots instead of their own LDS array. tests/test_brent_interleave.py must FAIL on this library (it passes
# on the shipped one); without the read-delay knob the variant usually passes, which is why the knob exists.
# Output: tools/vlib/alias.so (run with SHYFT_HIP_LIB=tools/vlib/alias.so). Run `make -C shyft_amd/csrc` first.
set -e
cd "$(dirname "$0")/../shyft_amd/csrc"
mkdir -p ../../tools/vlib
sed -e 's/jres\[j\] = GS_BRENT_JOB/jz1[j] = GS_BRENT_JOB/' -e 's/if (slot >= 0) z = jres\[slot\];/if (slot >= 0) z = jz1[slot];/' \
    kernels/ptgsk.hip > kernels/_ptgsk_alias.hip
n=$(grep -c "jz1\[j\] = GS_BRENT_JOB\|z = jz1\[slot\]" kernels/_ptgsk_alias.hip)
[ "$n" = 2 ] || { echo "alias patch did not apply ($n)"; rm -f kernels/_ptgsk_alias.hip; exit 1; }
others=$(ls _obj/*.o _obj/kernels/*.o | grep -v "kernels/ptgsk.o")
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -c kernels/_ptgsk_alias.hip -o /tmp/ptgsk_alias.o
rm -f kernels/_ptgsk_alias.hip
/opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared -o ../../tools/vlib/alias.so $others /tmp/ptgsk_alias.o -lrocblas -lrccl
echo built tools/vlib/alias.so
