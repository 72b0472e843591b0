#!/bin/bash
# r05 batch J: per-stack A/B (the library before the inline exp/log work vs the current per-stack choice), the
# calc_snow_state inline variant, then the whole GPU suite on the current library
set -o pipefail
R=$(pwd); mkdir -p gpurun_out
for st in "hbv_stack 524288" "pt_hs_k 1048576" "pt_ss_k 1048576" "pt_gs_k 1048576"; do
  set -- $st
  timeout -k 10 300 python tools/ptgsk_variants.py --stack $1 --cells $2 tools/vlib/pre.so shyft_amd/lib/libshyft_hip.so tools/vlib/pre.so shyft_amd/lib/libshyft_hip.so > gpurun_out/abj_$1.log 2>&1; rc=$?; echo "== $1"; cat gpurun_out/abj_$1.log
  case $rc in 124|134|137|139) exit $rc;; esac
done
timeout -k 10 300 python tools/ptgsk_variants.py shyft_amd/lib/libshyft_hip.so tools/vlib/csinl.so shyft_amd/lib/libshyft_hip.so tools/vlib/csinl.so > gpurun_out/var_j.log 2>&1; rc=$?; cat gpurun_out/var_j.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > gpurun_out/gputest_j.log 2>&1; rc=$?
tail -4 gpurun_out/gputest_j.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/gputest_j.log | head -20; exit $rc; }
echo BATCH_J_DONE
