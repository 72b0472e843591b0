#!/bin/bash
# r05 batch U: out-of-line dexp / dlog / dexp2 with SGPR-table constants (tc.so) vs the main build, every stack
set -o pipefail
mkdir -p gpurun_out
L=shyft_amd/lib/libshyft_hip.so
V=tools/vlib
for st in "hbv_stack 524288" "pt_hs_k 1048576" "pt_ss_k 1048576" "pt_gs_k 1048576"; do
  set -- $st
  timeout -k 10 300 python tools/ptgsk_variants.py --stack $1 --cells $2 $L $V/tc.so $L $V/tc.so > gpurun_out/abu_$1.log 2>&1; rc=$?; echo "== $1"; cat gpurun_out/abu_$1.log
  case $rc in 124|134|137|139) exit $rc;; esac
done
