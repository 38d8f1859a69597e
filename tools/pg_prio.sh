#!/usr/bin/env bash
# Pipelined-graph A/B: when the next view's geometry starts (run on the GPU box from the repo root)
set -euo pipefail
mkdir -p gpurun_out
export LSR_BENCH_RGB=0
for g in fwd start fwd start; do
    LSR_PG_GEO=$g timeout -k 10 150 python bench.py --no-cpu-baseline > gpurun_out/pg_$g.log 2>&1
    python3 - "$g" <<'PY'
import json, sys
p = sys.argv[1]
d = json.loads([l for l in open(f"gpurun_out/pg_{p}.log") if l.startswith("{")][-1])
print(p, d["ms_per_step_forms"])
PY
done
