"""The two streams' phase in the pipelined step, fast vs slow reps (measurement aid):

    python3 tools/pg_phase.py

bench.py's PipelinedGraphStep at C3.  Every graph launch of REPS reps x STEPS replays is bracketed by
timing events on its own stream (stream A: the step graph, stream B: the geometry graph), so per step
k we know when A ran step k and when B ran the geometry it launched in replay k.  Per rep: wall time
per step, A's busy fraction, B's busy fraction, B's duration per geometry, A's per step, and the
offset of B's start from A's start (the phase).
"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class _Timed:
    """A CUDAGraph wrapper whose replay() is bracketed by timing events on the current stream."""

    def __init__(self, graph, log, tag):
        self.graph, self.log, self.tag = graph, log, tag

    def replay(self):
        import torch
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        self.graph.replay()
        b.record()
        self.log.append((self.tag, a, b))


def main():
    import torch
    import bench
    from langsplat_amd.pipeline import PipelinedGraphStep
    from langsplat_amd.synthetic import CONFIGS, make_cameras, make_gaussians
    steps = int(os.environ.get("PH_STEPS", "200"))
    reps = int(os.environ.get("PH_REPS", "10"))
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
                            [model._language_feature], optim, model=model).capture()
    for _ in range(20):
        pg.replay()
    pg.synchronize()
    torch.cuda.synchronize()
    log = []
    pg.g_comp = [_Timed(g, log, "A") for g in pg.g_comp]
    # the wrapped graphs are launched by replay()'s Python path only (not lsr_graph_launch)
    import langsplat_amd.pipeline as _pipeline
    _pipeline._NATIVE_LAUNCH = False
    pg._launchers.clear()
    pg.g_geo = [_Timed(g, log, "B") for g in pg.g_geo]
    for rep in range(reps):
        time.sleep(0.02)
        log.clear()
        t0 = time.perf_counter()
        for _ in range(steps):
            pg.replay()
        pg.synchronize()
        torch.cuda.synchronize()
        wall = 1e3 * (time.perf_counter() - t0) / steps
        ref = log[0][1]
        A = [(ref.elapsed_time(a), ref.elapsed_time(b)) for tag, a, b in log if tag == "A"]
        B = [(ref.elapsed_time(a), ref.elapsed_time(b)) for tag, a, b in log if tag == "B"]
        n = min(len(A), len(B))
        skip = n // 5
        span = A[-1][1] - A[skip][0]
        a_busy = sum(e - s for s, e in A[skip:]) / span
        b_busy = sum(e - s for s, e in B[skip:n]) / (B[n - 1][1] - B[skip][0])
        a_dur = statistics.median(e - s for s, e in A[skip:])
        b_dur = statistics.median(e - s for s, e in B[skip:n])
        # B's graph launched in replay k vs A's step k start (both launched by replay k)
        phase = statistics.median(B[k][0] - A[k][0] for k in range(skip, n))
        lagB = statistics.median(B[k][0] - A[k - 1][1] for k in range(skip, n))
        print(f"rep {rep:2d}: {wall:.4f} ms/step  A busy {a_busy:.3f} dur {1e3 * a_dur:6.1f} us | "
              f"B busy {b_busy:.3f} dur {1e3 * b_dur:6.1f} us | B start - A start {1e3 * phase:7.1f} us, "
              f"B start - A(k-1) end {1e3 * lagB:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
