#!/bin/bash
# instruction-budget ablations: SQ counters per chunk of a 12-chunk calendar year for each variant library
set -o pipefail
for v in "$@"; do
  bash tools/r03_pmc.sh abl_$v "SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS" \
      python3 $(pwd)/tools/run_chunks.py $(pwd)/tools/variants/$v.so 1048576 12 || exit 1
done
echo ABL_DONE
