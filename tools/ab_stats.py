"""Side-by-side kernel average durations of two sets of rocprofv3 --stats runs (tools/ab_kernels.sh).

    python tools/ab_stats.py <dirs of A> -- <dirs of B>
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def load(dirs):
    acc = defaultdict(list)
    for d in dirs:
        if not os.path.isdir(d):
            continue
        for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                name = re.sub(r"^void ", "", row["Name"])[:60]
                acc[name].append(float(row["AverageNs"]) / 1e3)
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    i = sys.argv.index("--")
    a, b = load(sys.argv[1:i]), load(sys.argv[i + 1:])
    names = sorted(set(a) | set(b), key=lambda k: -max(a.get(k, 0), b.get(k, 0)))
    print("%-60s %9s %9s %7s" % ("kernel", "A us", "B us", "B/A"))
    for k in names:
        x, y = a.get(k, float("nan")), b.get(k, float("nan"))
        print("%-60s %9.2f %9.2f %7.3f" % (k, x, y, y / x if x else float("nan")))


if __name__ == "__main__":
    main()
