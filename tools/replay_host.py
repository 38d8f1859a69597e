"""Host time inside PipelinedGraphStep.replay(), by part (measurement aid, round 6):

    python3 tools/replay_host.py [--steps 300] [--sync]

bench.py's C3 language step as a PipelinedGraphStep; each stream-A and stream-B graph launch is wrapped
to time the host's hipGraphLaunch call, so the rest of replay() (its Python, events, stream waits) is
the difference.  --sync reads loss.item() after every replay (train.py:108).  Prints per replay: the
whole replay() call, the A launch, the B launch and the remainder (microseconds, medians).
"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class _Timed:
    def __init__(self, g, acc):
        self.g, self.acc = g, acc

    def replay(self):
        t0 = time.perf_counter_ns()
        self.g.replay()
        self.acc.append(time.perf_counter_ns() - t0)


def main():
    import torch
    import bench
    from langsplat_amd.pipeline import PipelinedGraphStep
    from langsplat_amd.synthetic import CONFIGS, make_cameras, make_gaussians
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 300
    sync = "--sync" in sys.argv
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
    for _ in range(50):
        pg.replay()
    torch.cuda.synchronize()
    la, lb, tot = [], [], []
    pg.g_comp = [_Timed(g, la) for g in pg.g_comp]
    # the wrapped graphs are launched by replay()'s Python path only (not lsr_graph_launch)
    import langsplat_amd.pipeline as _pipeline
    _pipeline._NATIVE_LAUNCH = False
    pg._launchers.clear()
    pg.g_geo = [_Timed(g, lb) for g in pg.g_geo]
    for _ in range(steps):
        t0 = time.perf_counter_ns()
        loss = pg.replay()
        tot.append(time.perf_counter_ns() - t0)
        if sync:
            loss.item()
    pg.synchronize()
    torch.cuda.synchronize()
    med = statistics.median
    a, b, t = med(la) / 1e3, med(lb) / 1e3, med(tot) / 1e3
    print(f"replay_host ({'synced' if sync else 'run-ahead'}): replay() {t:.1f} us, A graph launch {a:.1f} us, "
          f"B graph launch {b:.1f} us, the rest {t - a - b:.1f} us", flush=True)


if __name__ == "__main__":
    main()
