#!/bin/bash
# r04 batch: IDW row-group / occupancy variants (parity of two, kernel times of all), then the C5 measurement
set -o pipefail
R=$(pwd); mkdir -p gpurun_out
for v in g4w3 g2w4; do
  SHYFT_HIP_LIB=$R/tools/variants/$v.so timeout -k 10 300 python -u -m pytest tests/test_idw_c3.py tests/test_idw.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gt_e_$v.log 2>&1; rc=$?
  echo "parity $v rc=$rc"; tail -2 gpurun_out/gt_e_$v.log
  case $rc in 124|134|137|139) exit $rc;; esac
done
cd /tmp && export TMPDIR=/tmp
for v in c g4 g2w3 g4w3 g4w4 g2w4 g3w3 g4w2; do
  export SHYFT_HIP_LIB=$R/tools/variants/$v.so
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/idwe_$v -o run --output-format csv -- python3 $R/bench.py --idw --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/idwe_$v.log 2>&1 || { echo "PROF $v FAILED"; tail -5 $R/gpurun_out/idwe_$v.log; exit 1; }
  f=$(find $R/gpurun_out/idwe_$v -name "*kernel_stats.csv" | head -1); echo "== $v"; grep -i "idw_wave_gather" $f | cut -d, -f1-4
done
MB_LEAN=1 timeout -k 10 120 ./tools/mb/mb_brent tools/mb/jobs_jan.bin > gpurun_out/mb_lean.log 2>&1; cat gpurun_out/mb_lean.log
