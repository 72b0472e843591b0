#!/bin/bash
# round-3 PMC evidence: tools/gpu_profile.sh over several bench workloads in one GPU call, one gpurun_out/<tag>/
# per workload; usage: tools/r03_profile_all.sh tag1 tag2 ...  (tags below). Summaries are made afterwards with
# tools/pmc_summary.py --base gpurun_out/<tag> (see gpu_profile.sh).
set -o pipefail
for t in "$@"; do
  case $t in
    driver) A="--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"; K=ptgsk_run_kernel ;;
    default) A="--gpus 1 --steps 12 --warmup 1 --no-cpu-baseline"; K=ptgsk_run_kernel ;;
    hbv) A="--gpus 1 --stack hbv_stack --steps 12 --warmup 1 --no-cpu-baseline"; K=hbv_run_kernel ;;
    ptssk) A="--gpus 1 --stack pt_ss_k --steps 36 --warmup 1 --no-cpu-baseline"; K=ptssk_run_kernel ;;
    idw) A="--gpus 1 --idw --steps 12 --warmup 1 --no-cpu-baseline"; K=ptgsk_run_kernel ;;
    c131072) A="--gpus 1 --cells 131072 --steps 12 --warmup 1 --no-cpu-baseline"; K=ptgsk_run_kernel ;;
    *) echo "unknown tag $t"; exit 2 ;;
  esac
  echo "== $t: $A"
  TAG=$t BENCH_ARGS="$A" KERNEL=$K bash tools/gpu_profile.sh > gpurun_out/prof_$t.txt 2>&1 || { cat gpurun_out/prof_$t.txt; exit 1; }
  grep "prof .* ok" gpurun_out/prof_$t.txt | tr '\n' ' '; echo
done
echo PROFILE_ALL_DONE
