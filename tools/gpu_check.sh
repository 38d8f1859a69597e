#!/usr/bin/env bash
# GPU suite + bench runs (run on the GPU box from the repo root); outputs under gpurun_out/.
#   tools/gpu_check.sh [ab]   ab: also a bench with LSR_SPLIT_COLOR=1 (same-box A/B)
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 150 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1
if [ "${1:-}" = ab ]; then
    LSR_SPLIT_COLOR=1 timeout -k 10 150 python bench.py --no-cpu-baseline > gpurun_out/bench_splitcolor.log 2>&1
fi
timeout -k 10 150 python bench.py --no-cpu-baseline > gpurun_out/bench2.log 2>&1
