#!/usr/bin/env bash
# default bench (phase-based placement) x2 + the bucket timeline of a whole forward
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 bench.py --json-out gpurun_out/r21_bench_a.json > gpurun_out/r21_bench_a.log 2>&1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --json-out gpurun_out/r21_bench_b.json > gpurun_out/r21_bench_b.log 2>&1
timeout -k 10 200 python3 tools/bucket_timeline.py C3 > gpurun_out/r21_bucket_timeline.txt 2>&1
