#!/bin/bash
# r05 batch P: pt_ss_k with the SIMD-placed solver set up just before the step loop vs without (sslean7.so); the
# default bench line of this build
set -o pipefail
mkdir -p gpurun_out
L=shyft_amd/lib/libshyft_hip.so
V=tools/vlib
timeout -k 10 400 python tools/ptgsk_variants.py --stack pt_ss_k --cells 1048576 $V/sslean7.so $L $V/sslean7.so $L > gpurun_out/var_p_ss.log 2>&1; rc=$?
cat gpurun_out/var_p_ss.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 600 python bench.py > gpurun_out/bench_p.json 2> gpurun_out/bench_p.err; rc=$?
cut -c1-400 gpurun_out/bench_p.json
exit $rc
