#!/bin/bash
# r05 batch T: the Brent job with the prefix's log / exp interleaved with the first K series terms (K = 4, 6, 8)
set -o pipefail
mkdir -p gpurun_out
L=shyft_amd/lib/libshyft_hip.so
V=tools/vlib
timeout -k 10 400 python tools/ptgsk_variants.py $L $V/ilp4b.so $V/ilp8b.so $L $V/ilp4b.so $V/ilp8b.so > gpurun_out/var_t.log 2>&1; rc=$?
cat gpurun_out/var_t.log
exit $rc
