#!/bin/bash
# r05 batch R1: the whole GPU suite, smoke(), the driver's bench line (with cpu_baseline), the PMC passes of that command (library sha
# recorded) and the 131K-cell line, all on the current library
set -o pipefail
R=$(pwd); mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > gpurun_out/gputest_r.log 2>&1; rc=$?
tail -4 gpurun_out/gputest_r.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/gputest_r.log | head -20; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r.log 2>&1 || { tail -5 gpurun_out/smoke_r.log; exit 1; }
tail -1 gpurun_out/smoke_r.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r.json 2> gpurun_out/bench_r.err || { tail -5 gpurun_out/bench_r.err; exit 1; }
cut -c1-300 gpurun_out/bench_r.json
rm -rf gpurun_out/c2
ROUND=r05 TAG=c2 KERNEL=ptgsk_run_kernel BENCH_ARGS="--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline" bash tools/gpu_profile.sh || exit 1
timeout -k 10 200 python bench.py --cells 131072 --no-cpu-baseline > gpurun_out/bench_r_c131k.json 2> gpurun_out/bench_r_c131k.err || { tail -5 gpurun_out/bench_r_c131k.err; exit 1; }
cut -c1-250 gpurun_out/bench_r_c131k.json
echo BATCH_R1_DONE
