#!/bin/bash
# r04 batch: pt_gs_k parity of the default build (dead post-Brent calc_snow_state removed), variant timing against
# the previous build, the 1M and 131K bench lines
set -o pipefail
R=$(pwd); mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ptgsk_parity.py tests/test_ptgsk_instances.py tests/test_golden.py tests/test_region_kat.py tests/test_kat_ptgsk.py tests/test_fullsize_sampled.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gt_f.log 2>&1; rc=$?
tail -4 gpurun_out/gt_f.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 400 python tools/ptgsk_variants.py tools/variants/ptctl.so tools/variants/ptdead.so tools/variants/venq.so tools/variants/vlgc.so tools/variants/vlgcall.so tools/variants/ptctl.so > gpurun_out/var_f.log 2>&1; cat gpurun_out/var_f.log
timeout -k 10 300 python bench.py > gpurun_out/bench_f_1m.json 2> gpurun_out/bench_f_1m.err || { tail -5 gpurun_out/bench_f_1m.err; exit 1; }
cut -c1-400 gpurun_out/bench_f_1m.json
timeout -k 10 300 python bench.py --cells 131072 --no-cpu-baseline > gpurun_out/bench_f_131k.json 2> gpurun_out/bench_f_131k.err || { tail -5 gpurun_out/bench_f_131k.err; exit 1; }
cut -c1-400 gpurun_out/bench_f_131k.json
timeout -k 10 300 python tools/ptgsk_phases.py tools/variants/prof.so > gpurun_out/phases_f.log 2>&1; cat gpurun_out/phases_f.log
