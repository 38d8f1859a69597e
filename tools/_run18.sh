#!/usr/bin/env bash
# placed emission: kernel trace of the pipelined graph step + the bucket timeline (C3)
set -euo pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r18_trace -o t -- \
    python3 tools/step_trace.py pgraph > gpurun_out/r18_trace.log 2>&1
python3 tools/step_trace.py --timeline gpurun_out/r18_trace/t_kernel_trace.csv > gpurun_out/r18_timeline.txt
timeout -k 10 300 python3 tools/bucket_timeline.py C3 > gpurun_out/r18_bucket_timeline.txt 2>&1
