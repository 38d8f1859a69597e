"""Average PMC counters per kernel from a rocprofv3 --pmc CSV (measurement aid).

    python tools/pmc_show.py gpurun_out/<dir>/pmc_counter_collection.csv
"""
import csv
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    acc[r["Kernel_Name"][:48]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:30s} {sum(v) / len(v):.4g}  (n={len(v)})")
    if "SQ_LDS_IDX_ACTIVE" in d and "GRBM_GUI_ACTIVE" in d:
        g = sum(d["GRBM_GUI_ACTIVE"]) / len(d["GRBM_GUI_ACTIVE"]) / 8  # per XCD
        lds = sum(d["SQ_LDS_IDX_ACTIVE"]) / len(d["SQ_LDS_IDX_ACTIVE"])
        print(f"   LDS utilisation = {lds / (g * 256):.3f}")
