#!/bin/bash
# r05 first batch on the r04 kernels: PMC passes of the driver's command (C2) with the library sha recorded, then
# configs[4] per GPU at its horizon (pt_ss_k + routing, 1M cells x 26,280 steps = 60 chunks of 438) + its passes.
set -o pipefail
R=$(pwd); mkdir -p gpurun_out
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { echo C2 FAILED; tail -5 gpurun_out/bench_c2.err; exit 1; }
cut -c1-400 gpurun_out/bench_c2.json
ROUND=r05 TAG=c2 KERNEL=ptgsk_run_kernel BENCH_ARGS="--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline" bash tools/gpu_profile.sh || exit 1
timeout -k 10 600 python bench.py --gpus 1 --stack pt_ss_k --steps 60 --warmup 1 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || { echo C5 FAILED; tail -5 gpurun_out/bench_c5.err; exit 1; }
cut -c1-400 gpurun_out/bench_c5.json
ROUND=r05 TAG=c5 KERNEL=ptssk_run_kernel BENCH_ARGS="--gpus 1 --stack pt_ss_k --steps 60 --warmup 1 --no-cpu-baseline" bash tools/gpu_profile.sh || exit 1
echo BATCH_A_DONE
