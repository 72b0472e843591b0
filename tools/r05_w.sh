#!/bin/bash
# r05 batch W: pt_gs_k workgroups of 128 / 512 lanes with the SIMD-placed solver vs 256 (main)
set -o pipefail
mkdir -p gpurun_out
L=shyft_amd/lib/libshyft_hip.so
V=tools/vlib
timeout -k 10 400 python tools/ptgsk_variants.py $L $V/b128.so $V/b512.so $L $V/b128.so $V/b512.so > gpurun_out/var_w.log 2>&1; rc=$?
cat gpurun_out/var_w.log
exit $rc
