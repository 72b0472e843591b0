# A/B of the bench's forcing-generation modes (GPU box): ARGS are the bench arguments, MODES the --overlap-forcing values
mkdir -p gpurun_out/ov
for o in ${MODES:-0 -1 0 -1}; do
  n=ov$o.$RANDOM
  timeout -k 10 200 python3 bench.py ${ARGS:---gpus 1 --steps 20 --warmup 5} --no-cpu-baseline --overlap-forcing $o > gpurun_out/ov/$n.json 2> gpurun_out/ov/$n.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ov/$n.json')); print('overlap $o', '%.4g' % d['value'], round(d['ms_per_step'], 2), round(d['kernel_ms_per_step'], 2))"
done
