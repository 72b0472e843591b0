#!/bin/bash
# r05 batch O: the build with the trims, the SIMD-placed solver wavefront (pt_gs_k, pt_ss_k) and pt_ss_k's shared
# log + paired exp, against the r05 baseline library (pre.so) and the variant libraries it came from; then the
# whole GPU suite
set -o pipefail
mkdir -p gpurun_out
L=shyft_amd/lib/libshyft_hip.so
V=tools/vlib
timeout -k 10 400 python tools/ptgsk_variants.py $V/pre.so $L $V/rot3.so $L $V/rot3.so > gpurun_out/var_o.log 2>&1; rc=$?
cat gpurun_out/var_o.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 400 python tools/ptgsk_variants.py --stack pt_ss_k --cells 1048576 $V/pre.so $L $V/sslean7.so $L $V/sslean7.so > gpurun_out/var_o_ss.log 2>&1; rc=$?
cat gpurun_out/var_o_ss.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > gpurun_out/gputest_o.log 2>&1; rc=$?
tail -4 gpurun_out/gputest_o.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/gputest_o.log | head -20; exit $rc; }
echo BATCH_O_DONE
