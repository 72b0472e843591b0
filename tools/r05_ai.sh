#!/bin/bash
# r05 batch AI: Priestley-Taylor / Kirchner exp / log inline (per-call constant loads) in the other stacks
set -o pipefail
mkdir -p gpurun_out
L=shyft_amd/lib/libshyft_hip.so
V=tools/vlib
for st in "hbv_stack 524288 hbv" "pt_ss_k 1048576 ptssk" "pt_hs_k 1048576 pthsk" "pt_hps_k 1048576 pthpsk"; do
  set -- $st
  timeout -k 10 300 python tools/ptgsk_variants.py --stack $1 --cells $2 $L $V/ki_$3.so $L $V/ki_$3.so > gpurun_out/abai_$1.log 2>&1; rc=$?; echo "== $1"; cat gpurun_out/abai_$1.log
  case $rc in 124|134|137|139) exit $rc;; esac
done
