#!/usr/bin/env bash
# GPU shader clock (sysfs pp_dpm_sclk, the level marked *) sampled every ~20 ms while tools/pg_host.py
# runs six reps of 300 pipelined-graph steps: are the slow reps a lower clock?
set -uo pipefail
mkdir -p gpurun_out
out=gpurun_out/r22_clock.txt
: > $out
d=$(dirname "$(ls /sys/class/drm/card*/device/pp_dpm_sclk 2>/dev/null | head -1)")
echo "sysfs: ${d:-none}" >> $out
python3 - "$d" >> $out 2>&1 <<'PY' &
import os, sys, time
d = sys.argv[1]
t0 = time.time()
names = [n for n in ("pp_dpm_sclk", "pp_dpm_mclk", "pp_dpm_fclk", "pp_dpm_socclk") if os.path.exists(os.path.join(d, n))]
for _ in range(2500):
    row = []
    for n in names:
        try:
            cur = [l.split(":")[1].split()[0] for l in open(os.path.join(d, n)) if '*' in l]
        except Exception as e:
            cur = ["err"]
        row.append(f"{n[7:]}={cur[0] if cur else '-'}")
    print(f"{time.time():.3f} " + " ".join(row), flush=True)
    time.sleep(0.02)
PY
pid=$!
PG_HOST_REPS=12 timeout -k 10 200 python3 tools/pg_host.py --steps 300 > gpurun_out/r22_pgh.log 2>&1
rc=$?
kill $pid 2>/dev/null
wait $pid 2>/dev/null
exit $rc
