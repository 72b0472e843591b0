#!/bin/bash
# r05 batch I: A/B of the inline exp/log changes per stack on one box (the library before them vs the current one)
set -o pipefail
R=$(pwd); mkdir -p gpurun_out
for st in "hbv_stack 524288" "pt_ss_k 1048576" "pt_hs_k 1048576" "pt_gs_k 1048576"; do
  set -- $st
  timeout -k 10 300 python tools/ptgsk_variants.py --stack $1 --cells $2 tools/vlib/pre.so shyft_amd/lib/libshyft_hip.so tools/vlib/pre.so shyft_amd/lib/libshyft_hip.so > gpurun_out/ab_$1.log 2>&1; rc=$?; echo "== $1"; cat gpurun_out/ab_$1.log
  case $rc in 124|134|137|139) exit $rc;; esac
done
timeout -k 10 300 python tools/ptgsk_variants.py tools/vlib/base.so tools/vlib/csinl.so tools/vlib/slim.so tools/vlib/slimcs.so tools/vlib/base.so > gpurun_out/var_i.log 2>&1; rc=$?; cat gpurun_out/var_i.log
case $rc in 124|134|137|139) exit $rc;; esac
for lib in shyft_amd/lib/libshyft_hip.so tools/vlib/gen_nt.so shyft_amd/lib/libshyft_hip.so tools/vlib/gen_nt.so; do
  SHYFT_HIP_LIB=$R/$lib timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/gen.json 2>gpurun_out/gen.err || { tail -3 gpurun_out/gen.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/gen.json')); print('$lib', round(d['value']/1e9,3), round(d['ms_per_step'],2), round(d['kernel_ms_per_step'],2))"
done
echo BATCH_I_DONE
