#!/usr/bin/env bash
# Same-box A/B of an environment knob on the bench (run on the GPU box from the repo root):
#   tools/ab_env.sh VAR "valA valB" [rounds]  -> gpurun_out/ab_<VAR>_<val>_<round>.log
set -euo pipefail
var=$1
vals=$2
rounds=${3:-2}
mkdir -p gpurun_out
for r in $(seq 1 "$rounds"); do
    for v in $vals; do
        tag=$(basename "$v")
        env "$var=$v" timeout -k 10 120 python bench.py --no-cpu-baseline > "gpurun_out/ab_${var}_${tag}_${r}.log" 2>&1
    done
done
