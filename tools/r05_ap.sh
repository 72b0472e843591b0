#!/bin/bash
# r05 batch AP: the callee register budget of pt_gs_k's out-of-line functions (the never-launched budget kernel at
# 5 / 6 / 7 waves per SIMD instead of 8)
set -o pipefail
mkdir -p gpurun_out
L=shyft_amd/lib/libshyft_hip.so
V=tools/vlib
timeout -k 10 400 python tools/ptgsk_variants.py $L $V/bw5.so $V/bw4.so $V/bw3.so $L $V/bw5.so $V/bw4.so $V/bw3.so > gpurun_out/var_ap.log 2>&1; rc=$?
cat gpurun_out/var_ap.log
exit $rc
