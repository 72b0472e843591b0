#!/bin/bash
# r05 batch B: the sharded-region tests (combine-path self-check / fallbacks, threshold crossing, sample_cells), then
# configs[3] / configs[4] as stated on one GPU through 8 engine shards (tests + bench lines).
set -o pipefail
R=$(pwd); mkdir -p gpurun_out
: > gpurun_out/progress.log
timeout -k 10 600 python -u -m pytest tests/test_sharded.py tests/test_brent_interleave.py -x -v --timeout 300 --timeout-method thread > gpurun_out/t_sharded.log 2>&1; rc=$?
tail -25 gpurun_out/t_sharded.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 1500 python -u -m pytest tests/test_configs_sharded.py -x -v --timeout 1200 --timeout-method thread > gpurun_out/t_configs.log 2>&1; rc=$?
tail -8 gpurun_out/t_configs.log; cat gpurun_out/progress.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --stack hbv_stack --gpus 1 --shards 8 --total-cells 4194304 > gpurun_out/bench_c4_sh8.json 2> gpurun_out/bench_c4_sh8.err || { echo C4 FAILED; tail -5 gpurun_out/bench_c4_sh8.err; exit 1; }
cut -c1-300 gpurun_out/bench_c4_sh8.json
timeout -k 10 900 python bench.py --stack pt_ss_k --gpus 1 --shards 8 --total-cells 8388608 --steps 60 --warmup 1 > gpurun_out/bench_c5_sh8.json 2> gpurun_out/bench_c5_sh8.err || { echo C5 FAILED; tail -5 gpurun_out/bench_c5_sh8.err; exit 1; }
cut -c1-300 gpurun_out/bench_c5_sh8.json
echo BATCH_B_DONE
