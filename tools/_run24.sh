#!/usr/bin/env bash
# Adam step advance folded into the render backward: pipelined A/B (same library, LSR_BWD_ADVANCE)
set -euo pipefail
mkdir -p gpurun_out
rm -f gpurun_out/r24_pg.txt
for v in 1 0 1 0; do PG_HOST_REPS=8 LSR_BWD_ADVANCE=$v timeout -k 10 200 python3 tools/pg_host.py --steps 300 > gpurun_out/pgh.log 2>&1; echo "advance_in_bwd=$v $(grep 'summary' gpurun_out/pgh.log)" >> gpurun_out/r24_pg.txt; done
PG_HOST_REPS=4 LSR_LIB=langsplat_amd/liblsr_head.so timeout -k 10 200 python3 tools/pg_host.py --steps 300 > gpurun_out/pgh.log 2>&1; echo "head $(grep 'summary' gpurun_out/pgh.log)" >> gpurun_out/r24_pg.txt
