"""Issue-side utilisation of the bench kernels from the PMC passes of tools/pmc_valu.sh and
tools/pmc_lds.sh (measurement aid) -> profiles/<tag>_valu.json.

    python tools/valu_summary.py --sq gpurun_out/<tag>_sq/pmc_counter_collection.csv \
        --lds gpurun_out/<tag>_lds/pmc_counter_collection.csv --out profiles/<tag>_valu.json

valu_per_cu_cycle = SQ_INSTS_VALU / 256 CUs / (GRBM_GUI_ACTIVE / 8 XCDs): wave64 VALU instructions
issued per CU per cycle.  The CU's issue peak is ~2 (4 SIMDs x one wave64 VALU instruction per 2
cycles; tools/valu_peak.hip measures 1.85 for independent v_fma_f32 at 8 waves per SIMD,
profiles/r03_valu_peak.txt), so the VALU-issue fraction of the kernel's span is this / 2.  lds_utilisation =
SQ_LDS_IDX_ACTIVE / 256 CUs / (GRBM_GUI_ACTIVE / 8).
"""
import argparse
import csv
import json
import re
from collections import defaultdict

CUS, XCDS = 256, 8


def short(name):
    m = re.match(r"(?:void )?([\w:]+(?:<[^>]*>)?)", name)
    return m.group(1) if m else name


def load(path):
    acc = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sq", required=True)
    ap.add_argument("--lds")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    sq = load(a.sq)
    lds = load(a.lds) if a.lds else {}
    out = {}
    for k, d in sq.items():
        cyc = d.get("GRBM_GUI_ACTIVE", 0.0) / XCDS
        if not cyc:
            continue
        e = {"valu_insts": d.get("SQ_INSTS_VALU"), "salu_insts": d.get("SQ_INSTS_SALU"),
             "cycles": cyc, "valu_per_cu_cycle": d.get("SQ_INSTS_VALU", 0.0) / CUS / cyc}
        l = lds.get(k)
        if l and l.get("GRBM_GUI_ACTIVE"):
            e["lds_utilisation"] = l.get("SQ_LDS_IDX_ACTIVE", 0.0) / CUS / (l["GRBM_GUI_ACTIVE"] / XCDS)
        out[k] = e
    json.dump({"kernels": out}, open(a.out, "w"), indent=1, sort_keys=True)
    for k, e in out.items():
        print(f"{e['valu_per_cu_cycle']:.3f} VALU/CU-cycle  lds {e.get('lds_utilisation', float('nan')):.3f}  {k}")


if __name__ == "__main__":
    main()
