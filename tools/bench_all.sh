#!/bin/bash
# Every bench line of profiles/<round>, run from the repo root on the GPU box; outputs under gpurun_out/bench_all/.
# usage: tools/bench_all.sh [name ...]   (names: ptgsk hbv ptssk pthsk pthpsk idw btk dist2; default all but dist2)
# dist2 rehearses the 2-rank launcher path on a one-GPU box (gloo, both ranks on the one device).
set -e
O=gpurun_out/bench_all; mkdir -p $O
T="timeout -k 10 240"
names=${*:-"ptgsk hbv ptssk pthsk pthpsk idw btk"}
for n in $names; do
  case $n in
    ptgsk)  $T python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_ptgsk_n1.json 2> $O/e_$n.log ;;
    hbv)    $T python bench.py --stack hbv_stack > $O/bench_hbv_n1.json 2> $O/e_$n.log ;;
    ptssk)  $T python bench.py --stack pt_ss_k --steps 36 > $O/bench_ptssk_routing_36chunks_n1.json 2> $O/e_$n.log ;;
    pthsk)  $T python bench.py --stack pt_hs_k > $O/bench_pthsk_n1.json 2> $O/e_$n.log ;;
    pthpsk) $T python bench.py --stack pt_hps_k > $O/bench_pthpsk_n1.json 2> $O/e_$n.log ;;
    idw)    $T python bench.py --idw --no-cpu-baseline > $O/bench_idw_n1.json 2> $O/e_$n.log ;;
    btk)    $T python bench.py --btk --no-cpu-baseline > $O/bench_btk_n1.json 2> $O/e_$n.log ;;
    dist2)  SHYFT_DIST_BACKEND=gloo $T python bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline \
                > $O/bench_dist2_gloo_rehearsal.json 2> $O/e_$n.log ;;
    *) echo "unknown bench $n"; exit 2 ;;
  esac
done
echo done
