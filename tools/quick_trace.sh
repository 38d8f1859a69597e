#!/usr/bin/env bash
# Kernel trace of a short bench run (run on the GPU box from the repo root): gpurun_out/<tag>_qt/
set -euo pipefail
tag=${1:-qt}
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$(pwd)/gpurun_out/${tag}_qt" -o trace -- \
    python3 "$(pwd)/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "gpurun_out/${tag}_qt.log" 2>&1
