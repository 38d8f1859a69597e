"""Mean FETCH_SIZE / WRITE_SIZE per dispatch of the kernels matching a name filter, from a rocprofv3
--pmc counter_collection.csv (measurement aid; KB units as rocprofv3 reports them, converted to bytes):

    python3 tools/pmc_write_kernel.py <pmc_counter_collection.csv> <name substring>
"""
import csv
import sys
from collections import defaultdict


def main():
    path, sub = sys.argv[1], sys.argv[2]
    per = defaultdict(lambda: defaultdict(float))
    for row in csv.DictReader(open(path)):
        name = row.get("Kernel_Name", "")
        if sub not in name:
            continue
        per[(name, row.get("Dispatch_Id"))][row["Counter_Name"]] += float(row["Counter_Value"])
    agg = defaultdict(list)
    for (name, _), cs in per.items():
        for c, v in cs.items():
            agg[(name, c)].append(v)
    for (name, c), vs in sorted(agg.items()):
        print(f"{name[:70]:70s} {c:12s} dispatches {len(vs):3d} mean {sum(vs) / len(vs) * 1024 / 1e6:10.2f} MB")


if __name__ == "__main__":
    main()
