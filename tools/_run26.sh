#!/usr/bin/env bash
# loop alignment (-falign-loops) A/B on the pipelined step
set -euo pipefail
mkdir -p gpurun_out
rm -f gpurun_out/r26_pg.txt
for l in liblsr liblsr_al64 liblsr_al128 liblsr_al32 liblsr liblsr_al64 liblsr_al128 liblsr_al32; do PG_HOST_REPS=8 LSR_LIB=langsplat_amd/$l.so timeout -k 10 200 python3 tools/pg_host.py --steps 300 > gpurun_out/pgh.log 2>&1; echo "$l $(grep 'summary' gpurun_out/pgh.log)" >> gpurun_out/r26_pg.txt; done
