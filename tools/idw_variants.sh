#!/bin/bash
# Time the C3 interpolation (5 IDW gathers per 730-step chunk) for several libshyft_hip.so variants: the run
# kernel is the same in all of them, so the ms/step difference is the gathers. Usage: tools/idw_variants.sh lib.so...
for lib in "$@"; do
  SHYFT_HIP_LIB=$(realpath $lib) timeout -k 10 300 python bench.py --idw --steps 3 --warmup 1 --no-cpu-baseline \
    --no-catchment-sums | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$(basename $lib)', round(d['ms_per_step'],1), 'ms/step', round(d['ms_per_step']-d['kernel_ms_per_step'],1), 'ms outside the run kernel')"
done
