"""Where a synced step's extra time goes (measurement aid):

    python3 tools/sync_gap.py [--steps 200] [--spin]

(--spin: hipSetDeviceFlags(hipDeviceScheduleSpin) before the HIP runtime starts, i.e. the waiting
host thread spins instead of yielding)

train.py:108 reads loss.item() after every iteration.  With the pipelined graph (bench.py's
`pipelined_graph` form) that is `pg.replay().item()`: the host waits for the step, then enqueues
the next one, so stream A idles between the end of step k and the start of step k + 1.  This tool
wraps each stream-A step graph's replay with timing events (GPU) and perf_counter stamps (host) and
prints, per step (median over the timed steps):
  gap_gpu      stream A idle from the end of step k to the start of step k + 1 (events);
  host_item    the host's .item() call (enqueue of the copy + the wait for step k);
  host_pre     host time from .item()'s return to the graph launch call of step k + 1
               (replay()'s Python before the launch);
  launch_gpu   gap_gpu - host_pre: the wake-up of the waiting host plus the launch latency;
and the wall time per step of the synced loop and of the run-ahead loop (no .item()).
"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class _Timed:
    """A graph whose replay() records a timing event before and after it on the current stream."""

    def __init__(self, g, log):
        self.g, self.log = g, log

    def replay(self):
        import torch
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        self.log.append({"h_launch": time.perf_counter(), "a": a, "b": b})
        a.record()
        self.g.replay()
        b.record()


def main():
    if "--spin" in sys.argv:  # before anything initialises the HIP runtime
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        print("sync_gap: hipSetDeviceFlags(spin) ->", hip.hipSetDeviceFlags(1), flush=True)
    import torch
    import bench
    from langsplat_amd.pipeline import PipelinedGraphStep
    from langsplat_amd.synthetic import CONFIGS, make_cameras, make_gaussians
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 200
    c = CONFIGS["C3"]
    P, W, H = c["P"], c["width"], c["height"]
    dev = torch.device("cuda", 0)
    model = bench.Model(make_gaussians(P, seed=0).to(dev), include_feature=True)
    cam = make_cameras(1, W, H, device=dev)[0]
    bg = torch.zeros(3, device=dev)
    gen = torch.Generator().manual_seed(100)
    gt = torch.nn.functional.normalize(torch.randn((3, H, W), generator=gen), dim=0).to(dev)
    mask = (torch.rand((1, H, W), generator=gen) < 0.9).to(dev)
    optim = bench.AmdAdam([{"params": [model._language_feature], "lr": 0.0025, "name": "language_feature"}],
                          lr=0.0, eps=1e-15)
    pg = PipelinedGraphStep(lambda: bench.render(cam, model, bench.Pipe, bg, bench.Opt,
                                                 language_target=(gt, mask))["language_l1"],
                            [model._language_feature], optim).capture()
    for _ in range(200):
        pg.replay()
    pg.synchronize()
    torch.cuda.synchronize()
    # run-ahead wall time
    t0 = time.perf_counter()
    for _ in range(steps):
        pg.replay()
    pg.synchronize()
    torch.cuda.synchronize()
    ahead = 1e3 * (time.perf_counter() - t0) / steps
    log = []
    pg.g_comp = [_Timed(g, log) for g in pg.g_comp]
    if pg.g_comp0 is not None:
        pg.g_comp0 = _Timed(pg.g_comp0, log)
    for _ in range(20):
        pg.replay().item()
    torch.cuda.synchronize()
    log.clear()
    items = []
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = pg.replay()
        h1 = time.perf_counter()
        loss.item()
        items.append((h1, time.perf_counter()))
    torch.cuda.synchronize()
    synced = 1e3 * (time.perf_counter() - t0) / steps
    gap, pre, host_item, span = [], [], [], []
    for k in range(len(log) - 1):
        gap.append(1e3 * log[k]["b"].elapsed_time(log[k + 1]["a"]))
        span.append(1e3 * log[k]["a"].elapsed_time(log[k]["b"]))
        pre.append(1e6 * (log[k + 1]["h_launch"] - items[k][1]))
        host_item.append(1e6 * (items[k][1] - items[k][0]))
    med = statistics.median
    print(f"sync_gap: steps {steps}  run-ahead {ahead:.4f} ms/step  synced {synced:.4f} ms/step  "
          f"(+{1e3 * (synced - ahead):.1f} us)", flush=True)
    if not gap:  # the steady-state replays launch natively (lsr_graph_launch), past the timed wrapper
        print("sync_gap: per-step breakdown needs LSR_PG_NATIVE_LAUNCH=0", flush=True)
        return
    print(f"sync_gap: step graph on stream A {med(span):.1f} us; gap_gpu {med(gap):.1f} us "
          f"(p10 {sorted(gap)[len(gap) // 10]:.1f}, p90 {sorted(gap)[9 * len(gap) // 10]:.1f}); "
          f"host_item {med(host_item):.1f} us; host_pre {med(pre):.1f} us; "
          f"launch_gpu {med(gap) - med(pre):.1f} us", flush=True)


if __name__ == "__main__":
    main()
