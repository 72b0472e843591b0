#!/bin/bash
# r05 batch X: segment sums without the index array for identity segments; the whole GPU suite and the driver's
# bench line (its wall minus kernel time holds the segment sums)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > gpurun_out/gputest_x.log 2>&1; rc=$?
tail -4 gpurun_out/gputest_x.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/gputest_x.log | head -20; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_x -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/bench_x.json 2> $GRAFT_REPO_ROOT/gpurun_out/bench_x.err || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/bench_x.err; exit 1; }
cut -c1-300 $GRAFT_REPO_ROOT/gpurun_out/bench_x.json
echo BATCH_X_DONE
