set -e
for v in "LSR_ADAM_DEV_BLOCKS=512" "LSR_ADAM_DEV_BLOCKS=2048" "LSR_ADAM_DEV_BLOCKS=4096" "LSR_ADAM_ADVANCE=1"; do
  for rep in 1 2; do
    env $v LSR_BENCH_RGB=0 timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/ab_adam.log 2>&1
    echo "$v $(tail -1 gpurun_out/ab_adam.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["ms_per_step_eager"])')"
  done
done
