#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_sharded.py tests/test_bench_launch.py tests/test_capi.py tests/test_ptgsk_instances.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gt_b.log 2>&1; rc=$?
tail -12 gpurun_out/gt_b.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 500 python tools/ptgsk_variants.py tools/variants/ctl.so tools/variants/pruned2.so tools/variants/pruned3.so tools/variants/ctl.so > gpurun_out/var3.log 2>&1; cat gpurun_out/var3.log
