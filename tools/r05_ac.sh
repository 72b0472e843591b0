#!/bin/bash
# r05 batch AC: the paired-store generator -- parity against numpy, then the driver's bench command under
# rocprofv3 --kernel-trace --stats with the paired kernel (main) and the one-cell-per-lane kernel (gen1.so)
set -o pipefail
R=$(pwd); mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_generator.py tests/test_brent_interleave.py -x -v --timeout 200 --timeout-method thread > gpurun_out/t_gen.log 2>&1; rc=$?
tail -6 gpurun_out/t_gen.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
for v in main gen1; do
  if [ $v = gen1 ]; then export SHYFT_HIP_LIB=$R/tools/vlib/gen1.so; fi
  rm -rf $R/gpurun_out/prof_ac_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_ac_$v -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $R/gpurun_out/bench_ac_$v.json 2> $R/gpurun_out/bench_ac_$v.err || { tail -5 $R/gpurun_out/bench_ac_$v.err; exit 1; }
  cut -c1-200 $R/gpurun_out/bench_ac_$v.json
  grep -h "synthetic_forcing" $R/gpurun_out/prof_ac_$v/run_kernel_stats.csv | cut -c1-40,200-330
done
echo BATCH_AC_DONE
