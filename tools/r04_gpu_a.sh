set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_sharded.py tests/test_capi.py tests/test_bench_launch.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/sharded.log 2>&1; rc=$?
tail -15 gpurun_out/sharded.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python tools/ptgsk_phases.py tools/variants/prof.so > gpurun_out/phases.log 2>&1; cat gpurun_out/phases.log | tail -16
timeout -k 10 500 python tools/ptgsk_variants.py tools/variants/ctl.so tools/variants/w3.so tools/variants/rot.so > gpurun_out/var2.log 2>&1; cat gpurun_out/var2.log
