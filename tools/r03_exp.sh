#!/bin/bash
# round-3 experiment session (GPU box, repo root): the new regression tests, then pt_gs_k variant timings
# (tools/variants/*.so, bit-exact digest check) and phase profiles of the SHYFT_PROF builds.
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/exp; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "$TESTS" > $O/tests.log 2>&1
  rc=$?; tail -5 $O/tests.log; [ $rc -ne 0 ] && exit $rc
fi
if [ -n "$VARIANTS" ]; then
  timeout -k 10 ${VTIMEOUT:-600} python -u tools/ptgsk_variants.py ${VARGS} $VARIANTS > $O/variants.log 2>&1
  rc=$?; cat $O/variants.log; [ $rc -ne 0 ] && exit $rc
fi
for p in $PHASES; do
  timeout -k 10 300 python -u tools/ptgsk_phases.py $p > $O/phases_$(basename $p .so).log 2>&1
  rc=$?; echo "== $p"; cat $O/phases_$(basename $p .so).log; [ $rc -ne 0 ] && exit $rc
done
echo EXP_DONE
