set -e
rm -f gpurun_out/pgh_cap.txt
for l in liblsr liblsr_cap4096 liblsr liblsr_cap4096 liblsr liblsr_cap4096; do PG_HOST_REPS=6 LSR_LIB=langsplat_amd/$l.so timeout -k 10 200 python3 tools/pg_host.py --steps 300 > gpurun_out/pgh.log 2>&1; echo "$l $(grep 'summary' gpurun_out/pgh.log)" >> gpurun_out/pgh_cap.txt; done
