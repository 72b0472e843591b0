#!/bin/bash
# r04 batch d: pt_gs_k callee-budget variants and IDW pair-row variants (timing only; parity ran in batch c)
set -o pipefail
R=$(pwd); mkdir -p gpurun_out
timeout -k 10 500 python tools/ptgsk_variants.py tools/variants/ctl.so tools/variants/pin6.so tools/variants/pin8.so tools/variants/r04a.so > gpurun_out/var_d1.log 2>&1; cat gpurun_out/var_d1.log
cd /tmp && export TMPDIR=/tmp
for v in idwA idwC; do
  export SHYFT_HIP_LIB=$R/tools/variants/$v.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/idwprof_$v -o run --output-format csv -- python3 $R/bench.py --idw --chunk 730 --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/idwprof_$v.log 2>&1 || { echo "PROF $v FAILED"; tail -5 $R/gpurun_out/idwprof_$v.log; exit 1; }
  f=$(find $R/gpurun_out/idwprof_$v -name "*kernel_stats.csv" | head -1); echo "== $v"; grep -i "idw_wave_gather" $f | cut -d, -f1-4
done
