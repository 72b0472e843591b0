#!/bin/bash
# r05 batch F: Priestley-Taylor exp/log inline variants (hbv_stack at 512K cells, pt_gs_k at 1M), year in 730-chunks
set -o pipefail
R=$(pwd); mkdir -p gpurun_out
timeout -k 10 300 python tools/ptgsk_variants.py --stack hbv_stack --cells 524288 tools/vlib/hbv_base.so tools/vlib/hbv_ptinl.so > gpurun_out/var_f_hbv.log 2>&1; rc=$?; cat gpurun_out/var_f_hbv.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python tools/ptgsk_variants.py tools/vlib/base.so tools/vlib/ptinl.so > gpurun_out/var_f_pt.log 2>&1; rc=$?; cat gpurun_out/var_f_pt.log
case $rc in 124|134|137|139) exit $rc;; esac
echo BATCH_F_DONE
