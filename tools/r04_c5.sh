#!/bin/bash
# configs[4] per GPU at its horizon: pt_ss_k + routing, 1M cells x 26,280 steps (60 chunks of 438), bench line then
# the rocprofv3 passes of the same command
set -o pipefail
R=$(pwd); mkdir -p gpurun_out
timeout -k 10 600 python bench.py --gpus 1 --stack pt_ss_k --steps 60 --warmup 1 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || { echo C5 FAILED; tail -5 gpurun_out/bench_c5.err; exit 1; }
cut -c1-600 gpurun_out/bench_c5.json
ROUND=r04 TAG=c5 KERNEL=ptssk_run_kernel BENCH_ARGS="--gpus 1 --stack pt_ss_k --steps 60 --warmup 1 --no-cpu-baseline" bash tools/gpu_profile.sh || exit 1
echo C5_DONE
