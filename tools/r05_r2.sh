#!/bin/bash
# r05 batch R2: hbv_stack (C4 per GPU) and pt_ss_k (C5 horizon) bench lines with their PMC passes, and configs[4]
# as stated on one GPU through 8 engine shards, on the current library
set -o pipefail
R=$(pwd); mkdir -p gpurun_out
rm -rf gpurun_out/hbv gpurun_out/c5
ROUND=r05 TAG=hbv KERNEL=hbv_run_kernel BENCH_ARGS="--stack hbv_stack --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline" bash tools/gpu_profile.sh || exit 1
timeout -k 10 300 python bench.py --stack hbv_stack --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_r_hbv.json 2> gpurun_out/bench_r_hbv.err || { tail -5 gpurun_out/bench_r_hbv.err; exit 1; }
cut -c1-250 gpurun_out/bench_r_hbv.json
ROUND=r05 TAG=c5 KERNEL=ptssk_run_kernel BENCH_ARGS="--stack pt_ss_k --gpus 1 --steps 60 --warmup 1 --no-cpu-baseline" bash tools/gpu_profile.sh || exit 1
timeout -k 10 300 python bench.py --stack pt_ss_k --gpus 1 --steps 60 --warmup 1 --no-cpu-baseline > gpurun_out/bench_r_c5.json 2> gpurun_out/bench_r_c5.err || { tail -5 gpurun_out/bench_r_c5.err; exit 1; }
cut -c1-250 gpurun_out/bench_r_c5.json
timeout -k 10 600 python bench.py --stack pt_ss_k --gpus 1 --shards 8 --total-cells 8388608 --steps 60 --warmup 1 --no-cpu-baseline > gpurun_out/bench_r_c5_sh8.json 2> gpurun_out/bench_r_c5_sh8.err || { tail -5 gpurun_out/bench_r_c5_sh8.err; exit 1; }
cut -c1-250 gpurun_out/bench_r_c5_sh8.json
timeout -k 10 600 python bench.py --stack hbv_stack --gpus 1 --shards 8 --total-cells 4194304 --no-cpu-baseline > gpurun_out/bench_r_c4_sh8.json 2> gpurun_out/bench_r_c4_sh8.err || { tail -5 gpurun_out/bench_r_c4_sh8.err; exit 1; }
cut -c1-250 gpurun_out/bench_r_c4_sh8.json
timeout -k 10 300 python bench.py --idw --no-cpu-baseline > gpurun_out/bench_r_idw.json 2> gpurun_out/bench_r_idw.err || { tail -5 gpurun_out/bench_r_idw.err; exit 1; }
cut -c1-250 gpurun_out/bench_r_idw.json
echo BATCH_R2_DONE
