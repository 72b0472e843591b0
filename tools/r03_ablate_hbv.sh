#!/bin/bash
# hbv_stack instruction-budget ablations: SQ counters per chunk of the bench year for each variant library
set -o pipefail
for v in "$@"; do
  SHYFT_HIP_LIB=$(pwd)/tools/variants/hbv/$v.so bash tools/r03_pmc.sh hbv_$v "SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" \
      python3 $(pwd)/bench.py --stack hbv_stack --no-cpu-baseline --steps 12 --warmup 1 || exit 1
done
echo ABL_DONE
