#!/bin/bash
# r05 batch D: configs[3] / configs[4] as stated on one GPU through 8 engine shards (tests + bench lines)
set -o pipefail
R=$(pwd); mkdir -p gpurun_out
: > gpurun_out/progress.log
timeout -k 10 300 python -u -m pytest tests/test_sharded.py -x -v -s -k balance --timeout 240 --timeout-method thread > gpurun_out/t_balance.log 2>&1; rc=$?
grep -E "contiguous|balanced|PASS|FAIL|passed|failed" gpurun_out/t_balance.log | tail -6
[ $rc -eq 0 ] || { tail -30 gpurun_out/t_balance.log; exit $rc; }
timeout -k 10 1000 python -u -m pytest tests/test_configs_sharded.py -x -v --timeout 900 --timeout-method thread > gpurun_out/t_configs.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/t_configs.log | tail -8; cat gpurun_out/progress.log
[ $rc -eq 0 ] || { tail -30 gpurun_out/t_configs.log; exit $rc; }
timeout -k 10 300 python bench.py --stack hbv_stack --gpus 1 --shards 8 --total-cells 4194304 > gpurun_out/bench_c4_sh8.json 2> gpurun_out/bench_c4_sh8.err || { echo C4 FAILED; tail -5 gpurun_out/bench_c4_sh8.err; exit 1; }
cut -c1-300 gpurun_out/bench_c4_sh8.json
timeout -k 10 400 python bench.py --stack pt_ss_k --gpus 1 --shards 8 --total-cells 8388608 --steps 60 --warmup 1 > gpurun_out/bench_c5_sh8.json 2> gpurun_out/bench_c5_sh8.err || { echo C5 FAILED; tail -5 gpurun_out/bench_c5_sh8.err; exit 1; }
cut -c1-300 gpurun_out/bench_c5_sh8.json
echo BATCH_D_DONE
