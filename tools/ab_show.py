"""Summarise tools/ab_env.sh logs: ms/step, the stages and the step roofline per knob value."""
import glob
import json
import sys

var = sys.argv[1]
for f in sorted(glob.glob(f"gpurun_out/ab_{var}_*.log")):
    lines = [x for x in open(f) if x.startswith("{")]
    if not lines:
        print(f, "no result")
        continue
    d = json.loads(lines[-1])
    st = d["stages_ms_per_step"]
    print(f.split("/")[-1], d["ms_per_step"], "all-grads", d.get("ms_per_step_all_gradients"), "%.3e" % d["value"],
          " ".join(f"{k[:10]}={v * 1000:.1f}" for k, v in st.items()))
