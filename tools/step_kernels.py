"""Per-kernel durations of one bench step from a rocprofv3 kernel trace (measurement aid).

    python tools/step_kernels.py gpurun_out/<tag>_qt/trace_kernel_trace.csv [step index]
"""
import csv
import re
import sys


def short(n):
    m = re.match(r"(?:void )?([\w:]+(?:<[^>]*>)?)", n)
    return (m.group(1) if m else n)[:48]


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    idx = [i for i, r in enumerate(rows) if re.search(r"k_preprocess(?!_)", r["Kernel_Name"])]
    i0, i1 = idx[k], idx[k + 1]
    prev = None
    for r in rows[i0:i1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print("%-48s %8.2f us  gap %6.2f" % (short(r["Kernel_Name"]), (e - s) / 1e3, (s - prev) / 1e3 if prev else 0.0))
        prev = e
    print("step span %.2f us" % ((int(rows[i1]["Start_Timestamp"]) - int(rows[i0]["Start_Timestamp"])) / 1e3))


if __name__ == "__main__":
    main()
