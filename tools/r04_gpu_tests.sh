#!/bin/bash
# GPU tests given as arguments (default: the whole -m gpu suite), one pytest process, stops on a crash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest ${@:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1; rc=$?
tail -25 gpurun_out/gputest.log
exit $rc
