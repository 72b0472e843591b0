#!/bin/bash
# The round's bench lines and their rocprofv3 evidence in one parametrised runner (GPU box, from the repo root).
#
#   LINES="c2 c3 ..." [PROFILE="c2 c3 ..."] [ROUND=r06] bash tools/gpu_lines.sh
#
# Each name below is one bench.py command; LINES runs the bench line (gpurun_out/lines/<name>.json + .err), PROFILE
# runs tools/gpu_profile.sh on the same command (gpurun_out/lines/prof_<name>/: trace, FETCH, WRITE, SQ, VALU-class
# passes; the IDW line also its LDS pass) and records the library's sha256 there. The PMC summaries
# (profiles/<round>/pmc_*.json) are written afterwards on the CPU side from the pulled passes:
#   python3 tools/pmc_summary.py --kernel <kernel> --round r06 --bench-args "<args>" --base gpurun_out/lines/prof_<name>
# Every step runs under its own time limit and the script stops at the first failure.
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/lines
mkdir -p $OUT
declare -A ARGS KERN LIMIT
ARGS[c2]="--gpus 1 --steps 20 --warmup 5";                                   KERN[c2]=ptgsk_run_kernel;  LIMIT[c2]=300
ARGS[c2y]="--gpus 1";                                                        KERN[c2y]=ptgsk_run_kernel; LIMIT[c2y]=300
ARGS[c3]="--idw --steps 20 --warmup 1";                                      KERN[c3]=ptgsk_run_kernel;  LIMIT[c3]=400
ARGS[c4g]="--stack hbv_stack --steps 20 --warmup 5";                         KERN[c4g]=hbv_run_kernel;   LIMIT[c4g]=300
ARGS[c5h]="--stack pt_ss_k --steps 60 --warmup 1";                           KERN[c5h]=ptssk_run_kernel; LIMIT[c5h]=400
ARGS[c131k]="--cells 131072 --steps 20 --warmup 5 --no-cpu-baseline";        KERN[c131k]=ptgsk_run_kernel; LIMIT[c131k]=300
ARGS[c4s]="--stack hbv_stack --gpus 1 --shards 8 --total-cells 4194304 --steps 20 --warmup 1"; LIMIT[c4s]=600
ARGS[c5s]="--stack pt_ss_k --gpus 1 --shards 8 --total-cells 8388608 --steps 60 --warmup 1";   LIMIT[c5s]=900
ARGS[hs]="--stack pt_hs_k --steps 20 --warmup 1";                            KERN[hs]=pthsk_run_kernel;  LIMIT[hs]=300
ARGS[hps]="--stack pt_hps_k --steps 20 --warmup 1";                          KERN[hps]=pthpsk_run_kernel; LIMIT[hps]=300
ARGS[btk]="--btk --steps 20 --warmup 1 --no-cpu-baseline";                   KERN[btk]=ptgsk_run_kernel; LIMIT[btk]=600
python3 -c "from shyft_amd import _native; print(_native.lib_sha())" > $OUT/lib_sha.txt || exit 1
for name in $LINES; do
    [ -n "${ARGS[$name]}" ] || { echo "unknown line $name"; exit 1; }
    echo "line $name: python3 bench.py ${ARGS[$name]}"
    timeout -k 10 ${LIMIT[$name]} python3 bench.py ${ARGS[$name]} > $OUT/$name.json 2> $OUT/$name.err \
        || { echo "LINE $name FAILED"; tail -20 $OUT/$name.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$OUT/$name.json')); print('  value %.4g cell-steps/s, %.2f ms/step, kernel %.2f ms' % (d['value'], d['ms_per_step'], d['kernel_ms_per_step']))"
done
for name in $PROFILE; do
    [ -n "${KERN[$name]}" ] || { echo "no profile for $name"; exit 1; }
    echo "profile $name"
    LDS=""; [ "$name" = "c3" ] && LDS=1
    BENCH_ARGS="${ARGS[$name]}" KERNEL=${KERN[$name]} TAG=lines/prof_$name LDS_PASS=$LDS ROUND=${ROUND:-r06} \
        bash tools/gpu_profile.sh > $OUT/prof_$name.log 2>&1 || { echo "PROFILE $name FAILED"; tail -20 $OUT/prof_$name.log; exit 1; }
done
echo done
