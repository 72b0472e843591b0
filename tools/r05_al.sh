#!/bin/bash
# r05 batch AL: the driver's bench command, current library vs the previous profiled build (prev.so), alternated
set -o pipefail
R=$(pwd); mkdir -p gpurun_out
for rep in 1 2; do
  for v in main prev; do
    if [ $v = prev ]; then export SHYFT_HIP_LIB=$R/tools/vlib/prev.so; else unset SHYFT_HIP_LIB; fi
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_al_${v}_$rep.json 2> gpurun_out/bench_al_${v}_$rep.err || { tail -3 gpurun_out/bench_al_${v}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/bench_al_${v}_$rep.json')); print('$v', $rep, '%.4e' % d['value'], 'kernel %.2f' % d['kernel_ms_per_step'])"
  done
done
