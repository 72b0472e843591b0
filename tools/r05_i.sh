#!/bin/bash
# r05 batch I: A/B of the inline exp/log changes per stack on one box (the library before them vs the current one)
set -o pipefail
R=$(pwd); mkdir -p gpurun_out
for st in "hbv_stack 524288" "pt_ss_k 1048576" "pt_hs_k 1048576" "pt_gs_k 1048576"; do
  set -- $st
  timeout -k 10 300 python tools/ptgsk_variants.py --stack $1 --cells $2 tools/vlib/pre.so shyft_amd/lib/libshyft_hip.so tools/vlib/pre.so shyft_amd/lib/libshyft_hip.so > gpurun_out/ab_$1.log 2>&1; rc=$?; echo "== $1"; cat gpurun_out/ab_$1.log
  case $rc in 124|134|137|139) exit $rc;; esac
done
echo BATCH_I_DONE
