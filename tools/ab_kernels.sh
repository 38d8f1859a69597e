#!/usr/bin/env bash
# Same-box A/B of per-kernel average durations (run on the GPU box from the repo root):
#   bash tools/ab_kernels.sh <tag> <lib_a> <lib_b> [rounds]
# Each round traces a short bench run with each library (LSR_LIB) under rocprofv3 --kernel-trace
# --stats; tools/ab_stats.py prints the kernels' average durations side by side.
set -euo pipefail
tag=$1; a=$2; b=$3; rounds=${4:-2}
export TMPDIR=/tmp
for r in $(seq 1 "$rounds"); do
    for v in a b; do
        lib=$a; [ "$v" = b ] && lib=$b
        LSR_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
            -d "$(pwd)/gpurun_out/ab_${tag}_${v}${r}" -o trace -- \
            python3 "$(pwd)/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "gpurun_out/ab_${tag}_${v}${r}.log" 2>&1
    done
done
python3 tools/ab_stats.py gpurun_out/ab_${tag}_a* -- gpurun_out/ab_${tag}_b*
