#!/bin/bash
# r05 batch M: pt_ss_k sca_rel_red variants (1: inline exp/log + lean gamma, SGPR table; 2: shared log, out-of-line
# calls, out-of-line lean gamma; 5: exp-only SGPR table; 6: shared log only) vs the main build (pt_gs_k trims adopted);
# then the pt_gs_k phase profile of a SHYFT_PROF build
set -o pipefail
mkdir -p gpurun_out
L=shyft_amd/lib/libshyft_hip.so
V=tools/vlib
timeout -k 10 400 python tools/ptgsk_variants.py --stack pt_ss_k --cells 1048576 $L $V/sslean1.so $V/sslean2.so $V/sslean5.so $V/sslean6.so $L $V/sslean1.so $V/sslean2.so $V/sslean5.so $V/sslean6.so > gpurun_out/var_m_ss.log 2>&1; rc=$?
cat gpurun_out/var_m_ss.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python tools/ptgsk_phases.py $V/prof.so > gpurun_out/phases_m.log 2>&1; rc=$?
cat gpurun_out/phases_m.log
exit $rc
