#!/bin/bash
# hbv_stack bench line for each variant library built by tools/build_variants.sh hbv <dir> ... (run on the GPU
# box from the repo root): usage: hbv_variants.sh <dir>; the in-tree library first as the control.
set -o pipefail
mkdir -p gpurun_out/hbvvar
run() {
  timeout -k 10 240 python bench.py --stack hbv_stack --no-cpu-baseline --steps 12 --warmup 1 \
      > gpurun_out/hbvvar/$1.json 2> gpurun_out/hbvvar/$1.err || { echo "$1 FAILED rc=$?"; tail -5 gpurun_out/hbvvar/$1.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], '%.3e' % d['value'], 'ms/step %.2f' % d['ms_per_step'], 'kernel_ms', d['roofline'].get('kernel_ms', ''), 'frac %.3f' % d['roofline']['frac'])" gpurun_out/hbvvar/$1.json $1
}
run control || exit 1
for so in "$1"/*.so; do
  n=$(basename $so .so)
  SHYFT_HIP_LIB=$(realpath $so) run $n || exit 1
done
echo HBV_VARIANTS_DONE
