#!/bin/bash
# rocprofv3 evidence for the bench's dominant kernel, run from the repo root on the GPU box:
#  1. --kernel-trace --stats of the default bench (same command as the bench line, minus cpu_baseline)
#  2. separate --pmc passes (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE cannot share a pass)
#  3. one SQ pass (VALU instruction mix, wave cycles) for the fp64-VALU view of the kernel
# Outputs under gpurun_out/prof_*; the summaries worth keeping are copied into profiles/ by hand.
set -o pipefail
R=$(pwd)
ARGS=${BENCH_ARGS:-}
cd /tmp && export TMPDIR=/tmp
run() {  # name, extra rocprofv3 args..., then bench args after --
    local name=$1; shift
    timeout -k 10 600 rocprofv3 "$@" -d $R/gpurun_out/prof_$name -o run --output-format csv -- \
        python3 $R/bench.py --no-cpu-baseline $ARGS $BARGS > $R/gpurun_out/prof_$name.log 2>&1 \
        || { echo "PROF $name FAILED"; tail -20 $R/gpurun_out/prof_$name.log; exit 1; }
    echo "prof $name ok"
}
BARGS="--steps 12 --warmup 1" run trace --kernel-trace --stats
BARGS="--steps 12 --warmup 0" run fetch --kernel-trace --pmc FETCH_SIZE
BARGS="--steps 12 --warmup 0" run write --kernel-trace --pmc WRITE_SIZE
BARGS="--steps 12 --warmup 0" run sq --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE
cd $R
find gpurun_out -path "*prof_*" -name "*.csv" | sort
