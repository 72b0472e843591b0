#!/bin/bash
# rocprofv3 evidence for one bench line, run from the repo root on the GPU box. Every pass runs the SAME bench
# command ($BENCH_ARGS, default = the driver's `--gpus 1 --steps 20 --warmup 5`):
#  1. --kernel-trace --stats                (per-kernel durations; the line's kernel time must agree)
#  2. --kernel-trace --pmc FETCH_SIZE        (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE cannot share a pass)
#  3. --kernel-trace --pmc WRITE_SIZE
#  4. --kernel-trace --pmc SQ_*              (VALU issue: the bound that applies to the VALU-bound stacks)
#  5. --kernel-trace --pmc SQ_INSTS_VALU_*   (the VALU instructions by class: fp64 add / mul / fma / transcendental,
#                                             int32 / int64, conversions; the rest is moves, selects, lane reads)
#  6. (LDS_PASS=1) --kernel-trace --pmc SQ_LDS_*  (LDS bank conflicts of the IDW gathers)
# then tools/pmc_summary.py writes profiles/$ROUND/pmc_<workload>.json, the file bench.py reads for the same
# command's `traffic` / `valu` fields. Raw outputs stay under gpurun_out/prof_*; copy what is judged to profiles/.
set -o pipefail
R=$(pwd)
ARGS=${BENCH_ARGS:---gpus 1 --steps 20 --warmup 5}
ROUND=${ROUND:-r06}
KERNEL=${KERNEL:-ptgsk_run_kernel}
O=$R/gpurun_out/${TAG:-.}; mkdir -p $O   # TAG: one sub-directory per workload when a call profiles several
cd /tmp && export TMPDIR=/tmp
run() {  # name, rocprofv3 args...
    local name=$1; shift
    rm -rf $O/prof_$name
    timeout -k 10 400 rocprofv3 "$@" -d $O/prof_$name -o run --output-format csv -- \
        python3 $R/bench.py $ARGS > $O/prof_$name.log 2>&1 \
        || { echo "PROF $name FAILED"; tail -20 $O/prof_$name.log; exit 1; }
    echo "prof $name ok"
}
run trace --kernel-trace --stats
run fetch --kernel-trace --pmc FETCH_SIZE
run write --kernel-trace --pmc WRITE_SIZE
run sq --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE
run sqf --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT
if [ -n "$LDS_PASS" ]; then
  run lds --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS
fi
cd $R
echo "$ARGS" > $O/bench_args.txt
# build identity of the library these passes measured (bench.py only uses a summary with the same sha)
python3 -c "from shyft_amd import _native; print(_native.lib_sha())" > $O/lib_sha.txt || exit 1
echo "$KERNEL" > $O/kernel.txt
# the summary is written here after the call (profiles/ does not travel back from the box):
#   python3 tools/pmc_summary.py --kernel $KERNEL --round $ROUND --bench-args "$ARGS" --base $O
find $O -path "*prof_*" -name "*.csv" | sort
