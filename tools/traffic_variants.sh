#!/bin/bash
# HBM-side traffic of pt_gs_k (or pt_ss_k) kernel variants (GPU box, from the repo root): for each library, the 1M-cell bench
# region from Jan 1 through CHUNKS chunks of 730 steps (tools/run_chunks.py) under two rocprofv3 passes (FETCH_SIZE,
# WRITE_SIZE: they cannot share a pass), then the per-launch bytes of ptgsk_run_kernel (tools/traffic_summary.py).
#   [STACK=pt_ss_k] CHUNKS=2 bash tools/traffic_variants.sh lib1.so lib2.so ...
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/traffic; mkdir -p $O
CHUNKS=${CHUNKS:-2}
cd /tmp && export TMPDIR=/tmp
for lib in "$@"; do
    n=$(basename $lib .so)
    for c in FETCH_SIZE WRITE_SIZE; do
        rm -rf $O/${n}_$c
        timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c -d $O/${n}_$c -o run --output-format csv -- \
            python3 $R/tools/run_chunks.py $R/$lib 1048576 $CHUNKS ${STACK:-pt_gs_k} > $O/${n}_$c.log 2>&1 \
            || { echo "PASS $n $c FAILED"; tail -20 $O/${n}_$c.log; exit 1; }
    done
    python3 $R/tools/traffic_summary.py $O $n ${STACK:-pt_gs_k} || exit 1
done
