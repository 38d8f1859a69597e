#!/usr/bin/env bash
# placed emission on / off: the bench's forms (same library, same box)
set -euo pipefail
mkdir -p gpurun_out
for p in 1 0 1 0; do
  LSR_PLACED=$p timeout -k 10 300 python3 bench.py --no-cpu-baseline --json-out gpurun_out/r20_bench_p$p.json > gpurun_out/r20_bench.log 2>&1
  python3 -c "
import json; d=json.load(open('gpurun_out/r20_bench_p$p.json'))
print('placed=$p', d['ms_per_step'], d['ms_per_step_forms'], 'fwd_only', d['ms_forward_only'], 'depth', d['stages_ms_per_step']['depth order'], 'binning', d['stages_ms_per_step']['binning'])" >> gpurun_out/r20_summary.txt
done
