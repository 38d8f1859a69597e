#!/usr/bin/env bash
# placed emission: tests, bucket timelines, pipelined step A/B (LSR_PLACED=1 vs 0, same library)
set -euo pipefail
mkdir -p gpurun_out
tools/gpu_tests.sh r19_tests.log tests/test_gpu_binning.py tests/test_gpu_parity.py
timeout -k 10 200 python3 tools/bucket_timeline.py C3 > gpurun_out/r19_bt.txt 2>&1
LSR_LIB=langsplat_amd/liblsr_mb1.so LSR_BUCKET_MARK_BASE=2 timeout -k 10 200 python3 tools/bucket_timeline.py C3 > gpurun_out/r19_bt_mb.txt 2>&1
rm -f gpurun_out/r19_pg.txt
for p in 1 0 1 0; do PG_HOST_REPS=4 LSR_PLACED=$p timeout -k 10 200 python3 tools/pg_host.py --steps 300 > gpurun_out/pgh.log 2>&1; echo "placed=$p $(grep 'summary' gpurun_out/pgh.log)" >> gpurun_out/r19_pg.txt; done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r19_trace -o t -- \
    python3 tools/step_trace.py pgraph > gpurun_out/r19_trace.log 2>&1
python3 tools/step_trace.py --timeline gpurun_out/r19_trace/t_kernel_trace.csv > gpurun_out/r19_timeline.txt
