#!/usr/bin/env bash
# Selected GPU tests + one bench (run on the GPU box from the repo root); outputs under gpurun_out/.
#   tools/gpu_quick.sh "<pytest -k expression>"
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$1" > gpurun_out/gpu_quick.log 2>&1
timeout -k 10 150 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1
timeout -k 10 150 python bench.py --no-cpu-baseline > gpurun_out/bench2.log 2>&1
