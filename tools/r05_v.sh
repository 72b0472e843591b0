#!/bin/bash
# r05 batch V: pt_hps_k with the SGPR-table calls (tcall.so) vs the main build; the whole GPU suite on the main build
set -o pipefail
mkdir -p gpurun_out
L=shyft_amd/lib/libshyft_hip.so
V=tools/vlib
timeout -k 10 300 python tools/ptgsk_variants.py --stack pt_hps_k --cells 1048576 $L $V/tcall.so $L $V/tcall.so > gpurun_out/abv_hps.log 2>&1; rc=$?
cat gpurun_out/abv_hps.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > gpurun_out/gputest_v.log 2>&1; rc=$?
tail -4 gpurun_out/gputest_v.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/gputest_v.log | head -20; exit $rc; }
echo BATCH_V_DONE
