#!/usr/bin/env bash
# Profiling recipe for the bench workload (run on the GPU box from the repo root):
#   kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in separate PMC passes (they do not fit
#   one pass on gfx950, MI355X_MICROARCH.md "rocprofv3 PMC slots"), then a full bench line.
# Outputs go to gpurun_out/<tag>_*; tools/prof_summary.py turns them into profiles/<tag>_summary.json.
set -euo pipefail
tag=${1:-rNN}
root=$(pwd)
export TMPDIR=/tmp
out=$root/gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/${tag}_trace" -o trace -- \
    python3 "$root/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$out/${tag}_trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/${tag}_fetch" -o pmc -- \
    python3 "$root/bench.py" --steps 3 --warmup 2 --no-cpu-baseline > "$out/${tag}_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/${tag}_write" -o pmc -- \
    python3 "$root/bench.py" --steps 3 --warmup 2 --no-cpu-baseline > "$out/${tag}_write.log" 2>&1
