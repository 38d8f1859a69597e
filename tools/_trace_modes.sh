set -e
export TMPDIR=/tmp
for m in 0 1; do
  LSR_TRACE_NOWAIT=$m timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tm$m -o t -- python3 tools/step_trace.py pgraph > gpurun_out/tm$m.log 2>&1
done
