#!/bin/bash
# per-kernel times of the C3 line (bench --idw) for each IDW variant library: rocprofv3 --kernel-trace --stats
set -o pipefail
R=$(pwd); cd /tmp && export TMPDIR=/tmp
for lib in "$@"; do
  n=$(basename $lib .so)
  SHYFT_HIP_LIB=$R/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/idwprof_$n -o run --output-format csv -- \
      python3 $R/bench.py --idw --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/idwprof_$n.log 2>&1 || { echo "$n FAILED"; tail -5 $R/gpurun_out/idwprof_$n.log; exit 1; }
  echo "== $n"; python3 -c "
import csv,sys
for r in csv.DictReader(open('$R/gpurun_out/idwprof_$n/run_kernel_stats.csv')):
    if 'idw' in r['Name'] or 'ptgsk_run' in r['Name']: print('%-60s %6s calls %9.3f ms avg' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e6))
"
done
echo IDWPROF_DONE
