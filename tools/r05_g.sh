#!/bin/bash
# r05 batch G: kirchner / PT inline-exp pt_gs_k variants; the Brent solver microbenchmark (lean solver bit-identity on
# the 16,384 recorded January jobs, cycles per job at 1 / 1024 / 4096 wavefronts, 64 and 22 active lanes)
set -o pipefail
R=$(pwd); mkdir -p gpurun_out
timeout -k 10 400 python tools/ptgsk_variants.py tools/vlib/base.so tools/vlib/kinl.so tools/vlib/gsfinl.so tools/vlib/gsfkinl.so tools/vlib/lit.so tools/vlib/gsflit.so tools/vlib/kinllit.so tools/vlib/base.so > gpurun_out/var_g.log 2>&1; rc=$?; cat gpurun_out/var_g.log
case $rc in 124|134|137|139) exit $rc;; esac
MB_LEAN=1 timeout -k 10 120 ./tools/mb/mb_brent tools/mb/jobs_jan.bin > gpurun_out/mb_lean.log 2>&1; rc=$?; cat gpurun_out/mb_lean.log
case $rc in 124|134|137|139) exit $rc;; esac
echo BATCH_G_DONE
