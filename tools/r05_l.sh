#!/bin/bash
# r05 batch L: pt_gs_k trim levels 1-3 and pt_ss_k lean variants 1-3 against the main build
set -o pipefail
mkdir -p gpurun_out
L=shyft_amd/lib/libshyft_hip.so
V=tools/vlib
timeout -k 10 400 python tools/ptgsk_variants.py $L $V/trim.so $V/trim2.so $V/trim3.so $L $V/trim.so $V/trim2.so $V/trim3.so > gpurun_out/var_l.log 2>&1; rc=$?
cat gpurun_out/var_l.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 400 python tools/ptgsk_variants.py --stack pt_ss_k --cells 1048576 $L $V/sslean.so $V/sslean2.so $V/sslean3.so $L $V/sslean.so $V/sslean2.so $V/sslean3.so > gpurun_out/var_l_ss.log 2>&1; rc=$?
cat gpurun_out/var_l_ss.log
exit $rc
