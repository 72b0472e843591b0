#!/bin/bash
# r05 batch H: the current tree end to end -- the whole GPU suite, smoke(), the driver's bench line (with
# cpu_baseline), the PMC passes of that command (library sha recorded), the C5 horizon and C4-per-GPU lines
set -o pipefail
R=$(pwd); mkdir -p gpurun_out
: > gpurun_out/progress.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > gpurun_out/gputest_h.log 2>&1; rc=$?
tail -4 gpurun_out/gputest_h.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/gputest_h.log | head -20; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_h.log 2>&1 || { tail -5 gpurun_out/smoke_h.log; exit 1; }
tail -1 gpurun_out/smoke_h.log
timeout -k 10 300 python bench.py > gpurun_out/bench_h.json 2> gpurun_out/bench_h.err || { tail -5 gpurun_out/bench_h.err; exit 1; }
cut -c1-300 gpurun_out/bench_h.json
rm -rf gpurun_out/c2
ROUND=r05 TAG=c2 KERNEL=ptgsk_run_kernel BENCH_ARGS="--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline" bash tools/gpu_profile.sh || exit 1
timeout -k 10 300 python bench.py --stack pt_ss_k --steps 60 --warmup 1 --no-cpu-baseline > gpurun_out/bench_h_c5.json 2> gpurun_out/bench_h_c5.err || { tail -5 gpurun_out/bench_h_c5.err; exit 1; }
cut -c1-250 gpurun_out/bench_h_c5.json
timeout -k 10 300 python bench.py --stack hbv_stack --no-cpu-baseline > gpurun_out/bench_h_hbv.json 2> gpurun_out/bench_h_hbv.err || { tail -5 gpurun_out/bench_h_hbv.err; exit 1; }
cut -c1-250 gpurun_out/bench_h_hbv.json
echo BATCH_H_DONE
