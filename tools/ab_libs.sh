#!/usr/bin/env bash
# Same-box A/B of library builds on the bench step, alternating (measurement aid):
#   bash tools/ab_libs.sh <reps> <lib_a> <lib_b> [...]   (LSR_LIB per run; prints ms_per_step and stages)
set -e
reps=$1; shift
for r in $(seq 1 "$reps"); do
  for lib in "$@"; do
    LSR_LIB=$lib LSR_BENCH_RGB=0 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 > gpurun_out/ab_libs.log 2>&1
    echo "$(basename $lib) | $(tail -1 gpurun_out/ab_libs.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["stages_ms_per_step"]; r=d["pipelined_graph_reps_ms"]; print(d["ms_per_step"], "reps", r["min"], r["median"], "eager", d["ms_per_step_eager"], "sync", d["ms_per_step_with_sync"], "fwd-only", d["ms_forward_only"], "| depth", s["depth order"], "bin", s["binning"], "pre", s["preprocess"], "fwd", s["render forward"], "bwd", s["render backward"])')"
  done
done
