"""Prints step time, value and stage times of bench.py JSON lines (gpurun_out/bench*.log by default)."""
import glob
import json
import sys

for f in sys.argv[1:] or sorted(glob.glob("gpurun_out/bench*.log")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except (OSError, ValueError, IndexError) as e:
        print(f, "no result:", e)
        continue
    st = " ".join(f"{k}={v * 1e3:.1f}" for k, v in d.get("stages_ms_per_step", {}).items())
    print(f"{f}: {d['ms_per_step']:.4f} ms  {d['value']:.3e} {d['unit']}  [{st}]")
