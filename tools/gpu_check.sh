#!/usr/bin/env bash
# GPU suite + two bench runs (run on the GPU box from the repo root); outputs under gpurun_out/.
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1
timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/bench2.log 2>&1
