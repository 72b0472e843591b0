#!/bin/bash
# r04 batch: parity of the changed kernels, then timing of the variants against the pre-change builds
set -o pipefail
R=$(pwd); mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_idw.py tests/test_idw_c3.py tests/test_hbv_parity.py tests/test_pthsk.py tests/test_sharded.py tests/test_bench_launch.py tests/test_ptgsk_instances.py tests/test_capi.py tests/test_golden.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gt_c.log 2>&1; rc=$?
tail -6 gpurun_out/gt_c.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 400 python tools/ptgsk_variants.py tools/variants/ctl.so tools/variants/pruned2.so tools/variants/r04a.so > gpurun_out/var_c1.log 2>&1; cat gpurun_out/var_c1.log
timeout -k 10 300 python tools/ptgsk_variants.py --stack hbv_stack --cells 524288 tools/variants/pruned3.so tools/variants/r04a.so tools/variants/pruned3.so tools/variants/r04a.so > gpurun_out/var_c2.log 2>&1; cat gpurun_out/var_c2.log
cd /tmp && export TMPDIR=/tmp
for v in pruned3 r04a; do
  export SHYFT_HIP_LIB=$R/tools/variants/$v.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/idwprof_$v -o run --output-format csv -- python3 $R/bench.py --idw --chunk 730 --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/idwprof_$v.log 2>&1 || { echo "PROF $v FAILED"; tail -5 $R/gpurun_out/idwprof_$v.log; exit 1; }
  f=$(find $R/gpurun_out/idwprof_$v -name "*kernel_stats.csv" | head -1); echo "== $v"; grep -i "idw\|ptgsk" $f | cut -d, -f1-5 | head -12
done
