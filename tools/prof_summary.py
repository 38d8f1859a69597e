"""Summarise rocprofv3 outputs into profiles/: kernel time stats and PMC HBM traffic per launch.

    python tools/prof_summary.py --trace gpurun_out/prof/trace_kernel_trace.csv \
        --fetch gpurun_out/pmc_fetch/pmc_counter_collection.csv \
        --write gpurun_out/pmc_write/pmc_counter_collection.csv --out profiles/rNN_summary.json

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) reads half of the bytes of
a wide coalesced stream on gfx950 and is doubled; WRITE_SIZE (KiB) is taken as is.  Both are only
calibrated for 16-B-per-lane streaming access: treat other access shapes as estimates.
"""
import argparse
import csv
import json
import re
from collections import defaultdict


def short(name):
    m = re.match(r"(?:void )?([\w:]+(?:<[^>]*>)?)", name)
    return m.group(1) if m else name


def kernel_times(path):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        acc[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return {k: {"launches": len(v), "avg_us": sum(v) / len(v), "total_us": sum(v)} for k, v in acc.items()}


def counter(path, name):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == name:
            acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    out = {"kernels": {}}
    times = kernel_times(a.trace) if a.trace else {}
    fetch = counter(a.fetch, "FETCH_SIZE") if a.fetch else {}
    write = counter(a.write, "WRITE_SIZE") if a.write else {}
    for k in sorted(set(times) | set(fetch) | set(write)):
        d = dict(times.get(k, {}))
        if k in fetch:
            d["fetch_kib_raw"] = fetch[k]
            d["read_bytes"] = 2.0 * fetch[k] * 1024
        if k in write:
            d["write_kib"] = write[k]
            d["write_bytes"] = write[k] * 1024
        if k in fetch and k in write:
            d["hbm_bytes_per_launch"] = d["read_bytes"] + d["write_bytes"]
        out["kernels"][k] = d
    json.dump(out, open(a.out, "w"), indent=1, sort_keys=True)
    for k, d in sorted(out["kernels"].items(), key=lambda kv: -kv[1].get("total_us", 0))[:20]:
        print(f"{k:40s} n={d.get('launches', 0):4d} avg_us={d.get('avg_us', 0):9.1f} "
              f"hbm_MB={d.get('hbm_bytes_per_launch', 0) / 1e6:9.2f}")


if __name__ == "__main__":
    main()
