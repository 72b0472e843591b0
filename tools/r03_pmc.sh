#!/bin/bash
# PMC passes (one counter group per run) over a command; usage: tools/r03_pmc.sh NAME "counters;counters;..." cmd...
set -o pipefail
R=$(pwd); name=$1; groups=$2; shift 2
O=$R/gpurun_out/pmc_$name; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
IFS=';' read -ra G <<< "$groups"
for g in "${G[@]}"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $g -d $O/p$i -o run --output-format csv -- "$@" > $O/p$i.log 2>&1 \
    || { echo "PMC pass $i ($g) FAILED"; tail -5 $O/p$i.log; exit 1; }
  echo "pass $i ok: $g"
done
