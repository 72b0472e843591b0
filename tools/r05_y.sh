#!/bin/bash
# r05 batch Y: co-resident pt_gs_k workgroups started (TG_ID & 3) x STAGGER x 8K cycles apart (1, 3, 6)
set -o pipefail
mkdir -p gpurun_out
L=shyft_amd/lib/libshyft_hip.so
V=tools/vlib
timeout -k 10 400 python tools/ptgsk_variants.py $L $V/st1.so $V/st3.so $V/st6.so $L $V/st1.so $V/st3.so $V/st6.so > gpurun_out/var_y.log 2>&1; rc=$?
cat gpurun_out/var_y.log
exit $rc
