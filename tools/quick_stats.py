"""Print the headline fields of bench JSON files: value, ms/step and per-stage times."""
import json
import sys

for path in sys.argv[1:]:
    d = json.load(open(path))
    st = d.get("stages_ms_per_step", {})
    print(path, f"{d['value']:.4g}", d["ms_per_step"], d.get("raster_ms_per_step"),
          " ".join(f"{k}={v:.4g}" for k, v in st.items()))
