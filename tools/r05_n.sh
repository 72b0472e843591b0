#!/bin/bash
# r05 batch N: pt_gs_k Brent solver wavefront rotated over the workgroup's wavefronts (1: by block, 2: by block/8,
# 3: the wavefront on SIMD HW_ID.TG_ID & 3); pt_ss_k shared log (6) and shared log + paired exp (7)
set -o pipefail
mkdir -p gpurun_out
L=shyft_amd/lib/libshyft_hip.so
V=tools/vlib
timeout -k 10 400 python tools/ptgsk_variants.py $L $V/rot1.so $V/rot2.so $V/rot3.so $L $V/rot1.so $V/rot2.so $V/rot3.so > gpurun_out/var_n.log 2>&1; rc=$?
cat gpurun_out/var_n.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 400 python tools/ptgsk_variants.py --stack pt_ss_k --cells 1048576 $L $V/sslean6.so $V/sslean7.so $L $V/sslean6.so $V/sslean7.so > gpurun_out/var_n_ss.log 2>&1; rc=$?
cat gpurun_out/var_n_ss.log
exit $rc
