#!/bin/bash
# r05 batch AJ: hbv-physical-snow's exp / log inline (pt_hps_k, hpsi.so) and gs_front's exp / log inline (pt_gs_k,
# gsfi.so), both with per-call constant loads, vs main
set -o pipefail
mkdir -p gpurun_out
L=shyft_amd/lib/libshyft_hip.so
V=tools/vlib
timeout -k 10 300 python tools/ptgsk_variants.py --stack pt_hps_k --cells 1048576 $L $V/hpsi.so $L $V/hpsi.so > gpurun_out/var_aj_hps.log 2>&1; rc=$?; cat gpurun_out/var_aj_hps.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python tools/ptgsk_variants.py $L $V/gsfi.so $L $V/gsfi.so > gpurun_out/var_aj_gs.log 2>&1; rc=$?; cat gpurun_out/var_aj_gs.log
exit $rc
