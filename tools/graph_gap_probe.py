"""Idle time between consecutive HIP graphs on one stream (measurement aid), under the kernel trace:

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gap -o t -- python3 tools/graph_gap_probe.py
    python3 tools/graph_gap_probe.py --report gpurun_out/gap/t_kernel_trace.csv

Four forms, 50 repetitions each, every graph one ~40 us elementwise kernel on a 64 MB tensor:
  eager     the kernel launched eagerly, back to back
  graph     graph replays back to back
  graph_ev  graph replay, an event recorded after each
  graph_w   graph replay, an event recorded after each and the stream waiting on another stream's
            (long completed) event before each
  graph3    one graph holding three of the kernels (the gaps inside a graph, and between graphs)
The report prints the median gap between one kernel's end and the next one's start per form.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

FORMS = ("eager", "graph", "graph_ev", "graph_w", "graph3")
SCALES = {f: 1.0 + 0.001 * (i + 1) for i, f in enumerate(FORMS)}  # tells the forms apart in the trace


def run():
    import torch
    dev = torch.device("cuda", 0)
    x = torch.ones(16 << 20, device=dev)
    s = torch.cuda.Stream(dev)
    other = torch.cuda.Stream(dev)
    done = torch.cuda.Event()
    with torch.cuda.stream(other):
        torch.zeros(1, device=dev)
        done.record(other)
    torch.cuda.synchronize()
    graphs = {}
    s.wait_stream(torch.cuda.current_stream())
    for f in FORMS[1:]:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            x.mul_(SCALES[f])  # warm-up outside the capture
        with torch.cuda.graph(g, stream=s):
            for _ in range(3 if f == "graph3" else 1):
                x.mul_(SCALES[f])
        graphs[f] = g
    torch.cuda.synchronize()
    ev = torch.cuda.Event()
    for f in FORMS:
        with torch.cuda.stream(s):
            for _ in range(17 if f == "graph3" else 50):
                if f == "eager":
                    x.mul_(SCALES[f])
                    continue
                if f == "graph_w":
                    s.wait_event(done)
                graphs[f].replay()
                if f in ("graph_ev", "graph_w"):
                    ev.record(s)
        torch.cuda.synchronize()


def report(path):
    import csv
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    rows = [r for r in rows if "elementwise" in r["Kernel_Name"] or "mul" in r["Kernel_Name"].lower()]
    # the forms ran in order, 50 kernels each (plus the warm-ups): split by position
    n = len(rows)
    tail = rows[n - 4 * 50 - 51:]
    for i, f in enumerate(FORMS):
        seg = tail[50 * i:50 * (i + 1)] if f != "graph3" else tail[200:251]
        gaps = sorted((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(seg, seg[1:]))
        durs = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in seg)
        print(f"graph_gap {f:9s} median gap {gaps[len(gaps) // 2]:6.2f} us  (p90 {gaps[int(0.9 * len(gaps))]:6.2f})"
              f"  kernel {durs[len(durs) // 2]:6.2f} us")


if __name__ == "__main__":
    if "--report" in sys.argv:
        report(sys.argv[sys.argv.index("--report") + 1])
    else:
        run()
