#!/bin/bash
# r05 batch C: pt_gs_k variant timings (1M cells, the year in 12 chunks of 730, digests on both instances), then the
# parity tests of the current tree (sharded combine paths, interleaving, pt_gs_k parity / instances / KATs), then the
# racy alias variant must FAIL the interleaving test.
set -o pipefail
R=$(pwd); mkdir -p gpurun_out
timeout -k 10 600 python tools/ptgsk_variants.py tools/vlib/base.so tools/vlib/lean.so tools/vlib/spec4.so tools/vlib/leanspec4.so tools/vlib/b128.so tools/vlib/b128lean.so shyft_amd/lib/libshyft_hip.so > gpurun_out/var_c.log 2>&1; rc=$?; cat gpurun_out/var_c.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 700 python -u -m pytest tests/test_sharded.py tests/test_brent_interleave.py tests/test_ptgsk_parity.py tests/test_ptgsk_instances.py tests/test_kat_ptgsk.py -x -v --timeout 300 --timeout-method thread > gpurun_out/t_c.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/t_c.log | tail -40
[ $rc -eq 0 ] || exit $rc
SHYFT_HIP_LIB=$R/tools/vlib/alias.so timeout -k 10 200 python -u -m pytest tests/test_brent_interleave.py -x -q --timeout 150 --timeout-method thread -k delayed > gpurun_out/t_alias.log 2>&1; rc=$?
tail -3 gpurun_out/t_alias.log; echo "alias variant pytest rc=$rc (1 = the test caught the race)"
case $rc in 124|134|137|139) exit $rc;; esac
echo BATCH_C_DONE
