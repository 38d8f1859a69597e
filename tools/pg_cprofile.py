"""Host-side profile of PipelinedGraphStep.replay (measurement aid):

    python3 tools/pg_cprofile.py [--sync]

bench.py's pipelined graph step at C3; 300 replays under cProfile (--sync: loss.item() after every
replay, train.py:108's pattern), top functions by own time, and the per-replay host time.
"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from langsplat_amd.pipeline import PipelinedGraphStep
    from langsplat_amd.synthetic import CONFIGS, make_cameras, make_gaussians
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
    sync = "--sync" in sys.argv
    for _ in range(30):
        pg.replay()
    torch.cuda.synchronize()
    n = 300
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    for _ in range(n):
        loss = pg.replay()
        if sync:
            loss.item()
    pr.disable()
    pg.synchronize()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    print(f"{'synced' if sync else 'run-ahead'}: {1e3 * (t1 - t0) / n:.4f} ms per replay (under cProfile)")
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
