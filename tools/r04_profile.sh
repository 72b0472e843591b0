#!/bin/bash
# r04 rocprofv3 evidence: kernel trace + FETCH / WRITE / SQ passes (tools/gpu_profile.sh) for the three bench lines
set -o pipefail
R=$(pwd)
ROUND=r04 TAG=c2 KERNEL=ptgsk_run_kernel BENCH_ARGS="--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline" bash tools/gpu_profile.sh || exit 1
ROUND=r04 TAG=hbv KERNEL=hbv_run_kernel BENCH_ARGS="--gpus 1 --stack hbv_stack --steps 20 --warmup 1 --no-cpu-baseline" bash tools/gpu_profile.sh || exit 1
ROUND=r04 TAG=c3 KERNEL=ptgsk_run_kernel BENCH_ARGS="--gpus 1 --idw --steps 20 --warmup 1 --no-cpu-baseline" bash tools/gpu_profile.sh || exit 1
echo PROFILE_DONE
