#!/usr/bin/env bash
# Same-box A/B of runtime environment variants on the bench step (measurement aid):
#   bash tools/ab_env.sh "VAR=1" "VAR=0 OTHER=2" ...   (each variant twice; prints ms_per_step, eager)
set -e
for v in "$@"; do
  for rep in 1 2; do
    env $v LSR_BENCH_RGB=0 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 > gpurun_out/ab_env.log 2>&1
    echo "$v | $(tail -1 gpurun_out/ab_env.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["stages_ms_per_step"]; print(d["ms_per_step"], d["ms_per_step_eager"], d["ms_per_step_with_sync"], "depth", s["depth order"], "bin", s["binning"], "adam", s["adam"], "fwd", s["render forward"], "bwd", s["render backward"])')"
  done
done
