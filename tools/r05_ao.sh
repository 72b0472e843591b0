#!/bin/bash
# r05 batch AO: the final library's pt_hs_k and pt_hps_k lines, and the driver's C2 command twice more (box spread)
set -o pipefail
mkdir -p gpurun_out
for st in pt_hs_k pt_hps_k; do
  timeout -k 10 300 python bench.py --stack $st --no-cpu-baseline > gpurun_out/bench_ao_$st.json 2> gpurun_out/bench_ao_$st.err || { tail -3 gpurun_out/bench_ao_$st.err; exit 1; }
  cut -c1-160 gpurun_out/bench_ao_$st.json
done
for rep in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_ao_c2_$rep.json 2> gpurun_out/bench_ao_c2_$rep.err || { tail -3 gpurun_out/bench_ao_c2_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_ao_c2_$rep.json')); print('C2 rep $rep', '%.4e' % d['value'], 'kernel %.2f' % d['kernel_ms_per_step'], 'traffic', d['roofline']['traffic'])"
done
