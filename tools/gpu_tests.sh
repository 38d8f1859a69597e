#!/usr/bin/env bash
# Selected GPU test files on the GPU box (from the repo root); log under gpurun_out/.
#   tools/gpu_tests.sh <log-name> <pytest args...>
set -euo pipefail
mkdir -p gpurun_out
log=gpurun_out/$1
shift
timeout -k 10 1000 python -u -m pytest -x -v --timeout 400 --timeout-method thread --durations=15 -m gpu "$@" > "$log" 2>&1
