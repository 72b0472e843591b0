set -e
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/kt; cd /tmp; export TMPDIR=/tmp
for s in hbv_stack pt_ss_k pt_hs_k pt_gs_k; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/kt/$s -o run -- python3 $R/bench.py --stack $s --no-routing --no-cpu-baseline --steps 2 --warmup 0 > $R/gpurun_out/kt/$s.log 2>&1
done
echo ok
