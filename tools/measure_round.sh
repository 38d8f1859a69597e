#!/usr/bin/env bash
# The round's measurements on the GPU box (from the repo root); everything under gpurun_out/:
#   tools/measure_round.sh r04
#   1. bench.py (C3, CPU baseline included)                  -> <tag>_bench.json / .log
#   2. kernel trace of the pipelined graph step (C3)         -> <tag>_pg_trace/, <tag>_pg_timeline.txt
#   3. tools/profile_round.sh <tag> C3 (trace + PMC passes)  -> <tag>_C3_{kernel_stats.csv,summary,valu}.json
set -euo pipefail
tag=${1:-rNN}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py --json-out gpurun_out/${tag}_bench.json > gpurun_out/${tag}_bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${tag}_pg_trace -o t -- \
    python3 tools/step_trace.py pgraph > gpurun_out/${tag}_pg_trace.log 2>&1
python3 tools/step_trace.py --timeline gpurun_out/${tag}_pg_trace/t_kernel_trace.csv > gpurun_out/${tag}_pg_timeline.txt
tools/profile_round.sh ${tag} C3
