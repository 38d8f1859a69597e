#!/usr/bin/env bash
# kernel stats of the pipelined step: current library vs liblsr_head.so
set -euo pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r25_new -o t -- \
    python3 tools/step_trace.py pgraph > gpurun_out/r25_new.log 2>&1
LSR_LIB=langsplat_amd/liblsr_head.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r25_head -o t -- \
    python3 tools/step_trace.py pgraph > gpurun_out/r25_head.log 2>&1
