#!/usr/bin/env bash
# buffer sets of the pipelined graph: 3 (default) vs 4
set -euo pipefail
mkdir -p gpurun_out
rm -f gpurun_out/r27_pg.txt
for n in 3 4 3 4; do PG_HOST_REPS=8 LSR_PG_SETS=$n timeout -k 10 200 python3 tools/pg_host.py --steps 300 > gpurun_out/pgh.log 2>&1; echo "sets=$n $(grep 'summary' gpurun_out/pgh.log)" >> gpurun_out/r27_pg.txt; done
