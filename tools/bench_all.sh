set -e
O=gpurun_out/r01b; mkdir -p $O
T="timeout -k 10 240"
$T python bench.py > $O/bench_n1.json 2> $O/e1.log
$T python bench.py --stack hbv_stack --cpu-cells 4000 > $O/bench_hbv_n1.json 2> $O/e2.log
$T python bench.py --stack pt_ss_k > $O/bench_ptssk_routing_n1.json 2> $O/e3.log
$T python bench.py --stack pt_hs_k > $O/bench_pthsk_n1.json 2> $O/e4.log
$T python bench.py --stack pt_hps_k > $O/bench_pthpsk_n1.json 2> $O/e5.log
$T python bench.py --idw --no-cpu-baseline > $O/bench_idw_n1.json 2> $O/e6.log
$T python bench.py --btk --no-cpu-baseline > $O/bench_btk_n1.json 2> $O/e7.log
echo done
