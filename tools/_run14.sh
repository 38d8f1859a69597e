set -e
export TMPDIR=/tmp
timeout -k 10 400 bash tools/ab_kernels.sh prent langsplat_amd/liblsr.so langsplat_amd/liblsr_prent.so 2 > gpurun_out/ab_prent.txt 2>&1
rm -f gpurun_out/pgh_nt.txt
for l in liblsr liblsr_prent liblsr liblsr_prent; do LSR_LIB=langsplat_amd/$l.so timeout -k 10 200 python3 tools/pg_host.py --steps 300 > gpurun_out/pgh.log 2>&1; echo "$l $(grep 'rep 2' gpurun_out/pgh.log)" >> gpurun_out/pgh_nt.txt; done
bash tools/_trace_modes.sh
