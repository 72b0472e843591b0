#!/bin/bash
# r05 batch K: pt_gs_k live-range trims (carry dead across the Brent phase, one storage field; forcing reload) and
# pt_ss_k's lean sca_rel_red (shared log of the two pdfs, inline exp / log, lean full-precision gamma) vs the main build
set -o pipefail
mkdir -p gpurun_out
L=shyft_amd/lib/libshyft_hip.so
timeout -k 10 400 python tools/ptgsk_variants.py $L tools/vlib/trim.so tools/vlib/trimrl.so $L tools/vlib/trim.so tools/vlib/trimrl.so > gpurun_out/var_k.log 2>&1; rc=$?
cat gpurun_out/var_k.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 400 python tools/ptgsk_variants.py --stack pt_ss_k --cells 1048576 $L tools/vlib/sslean.so $L tools/vlib/sslean.so > gpurun_out/var_k_ss.log 2>&1; rc=$?
cat gpurun_out/var_k_ss.log
exit $rc
