#!/usr/bin/env bash
# counter reduction workgroup size: pipelined step A/B (same box)
set -euo pipefail
mkdir -p gpurun_out
rm -f gpurun_out/r23_pg.txt
for l in liblsr liblsr_pub256 liblsr_pub512 liblsr liblsr_pub256 liblsr_pub512; do PG_HOST_REPS=8 LSR_LIB=langsplat_amd/$l.so timeout -k 10 200 python3 tools/pg_host.py --steps 300 > gpurun_out/pgh.log 2>&1; echo "$l $(grep 'summary' gpurun_out/pgh.log)" >> gpurun_out/r23_pg.txt; done
