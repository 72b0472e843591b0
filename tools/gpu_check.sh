#!/bin/bash
# One GPU session from the repo root: the -m gpu suite, then (unless the suite crashed or hung) the default
# bench line and any extra bench lines in $BENCH_EXTRA (';'-separated argument lists).
# Test failures do not stop the bench; a crash / abort / timeout (124, 134, 137, 139) stops everything.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
crashed() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-700} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
      ${TEST_ARGS} > gpurun_out/gputest.log 2>&1
  rc=$?
  tail -4 gpurun_out/gputest.log
  if crashed $rc; then echo "GPU TESTS CRASHED rc=$rc"; exit $rc; fi
  [ $rc -ne 0 ] && grep -E "FAILED|Error" gpurun_out/gputest.log | head -20
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?
  cat gpurun_out/bench.json
  if [ $rc -ne 0 ]; then echo "BENCH FAILED rc=$rc"; tail -20 gpurun_out/bench.err; exit $rc; fi
fi
if [ -n "$BENCH_EXTRA" ]; then
  i=0
  IFS=';' read -ra LINES <<< "$BENCH_EXTRA"
  for args in "${LINES[@]}"; do
    i=$((i+1))
    timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py $args > gpurun_out/bench_x$i.json 2> gpurun_out/bench_x$i.err
    rc=$?
    echo "== $args"; cat gpurun_out/bench_x$i.json
    if [ $rc -ne 0 ]; then echo "BENCH '$args' FAILED rc=$rc"; tail -20 gpurun_out/bench_x$i.err; exit $rc; fi
  done
fi
echo GPU_CHECK_DONE
