#!/bin/bash
# r04 batch: pt_gs_k workgroup-size variants, the Brent solver microbenchmark, IDW row-group / occupancy variants
set -o pipefail
R=$(pwd); mkdir -p gpurun_out
timeout -k 10 420 python tools/ptgsk_variants.py tools/variants/base.so tools/variants/b128.so tools/variants/b128s.so tools/variants/b64w4.so tools/variants/base.so > gpurun_out/var_g.log 2>&1; rc=$?; cat gpurun_out/var_g.log
case $rc in 124|134|137|139) exit $rc;; esac
MB_LEAN=1 timeout -k 10 120 ./tools/mb/mb_brent tools/mb/jobs_jan.bin > gpurun_out/mb_lean.log 2>&1; rc=$?; cat gpurun_out/mb_lean.log
case $rc in 124|134|137|139) exit $rc;; esac
cd /tmp && export TMPDIR=/tmp
for v in c g4 g2w3 g4w3 g4w4 g2w4; do
  export SHYFT_HIP_LIB=$R/tools/variants/$v.so
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/idwe_$v -o run --output-format csv -- python3 $R/bench.py --idw --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/idwe_$v.log 2>&1 || { echo "PROF $v FAILED"; tail -5 $R/gpurun_out/idwe_$v.log; exit 1; }
  f=$(find $R/gpurun_out/idwe_$v -name "*kernel_stats.csv" | head -1); echo "== $v"; grep -i "idw_wave_gather" $f | cut -d, -f1-4
done
