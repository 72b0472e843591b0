#!/bin/bash
# r05 batch E: pt_gs_k 512-lane workgroups vs the default, IDW row-group variants (rocprofv3 per-kernel times of the
# C3 gathers), the 131K-cell shard line, and the C2 line with the generator overlapped (no CU mask).
set -o pipefail
R=$(pwd); mkdir -p gpurun_out
timeout -k 10 300 python tools/ptgsk_variants.py tools/vlib/base.so tools/vlib/b512.so tools/vlib/u2.so tools/vlib/u2b512.so shyft_amd/lib/libshyft_hip.so > gpurun_out/var_e.log 2>&1; rc=$?; cat gpurun_out/var_e.log
case $rc in 124|134|137|139) exit $rc;; esac
cd /tmp && export TMPDIR=/tmp
for v in idw_c idw_g4 idw_g2w3 idw_g4w3 idw_g2w3z idw_g4w4z; do
  export SHYFT_HIP_LIB=$R/tools/vlib/$v.so
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/idwe_$v -o run --output-format csv -- python3 $R/bench.py --idw --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/idwe_$v.log 2>&1 || { echo "PROF $v FAILED"; tail -5 $R/gpurun_out/idwe_$v.log; exit 1; }
  f=$(find $R/gpurun_out/idwe_$v -name "*kernel_stats.csv" | head -1); echo "== $v"; grep -i "idw_wave_gather" $f | cut -d, -f1-4
done
unset SHYFT_HIP_LIB
cd $R
timeout -k 10 200 python bench.py --cells 131072 --no-cpu-baseline > gpurun_out/bench_c131k.json 2> gpurun_out/bench_c131k.err || { echo 131K FAILED; tail -5 gpurun_out/bench_c131k.err; exit 1; }
cut -c1-250 gpurun_out/bench_c131k.json
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_c2_new.json 2> gpurun_out/bench_c2_new.err || { echo C2 FAILED; tail -5 gpurun_out/bench_c2_new.err; exit 1; }
cut -c1-250 gpurun_out/bench_c2_new.json
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --overlap-forcing -1 > gpurun_out/bench_c2_ovl.json 2> gpurun_out/bench_c2_ovl.err || { echo OVL FAILED; tail -5 gpurun_out/bench_c2_ovl.err; exit 1; }
cut -c1-250 gpurun_out/bench_c2_ovl.json
echo BATCH_E_DONE
