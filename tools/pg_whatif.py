"""What bounds the pipelined step (measurement aid; results of the shortened forms are NOT valid):

    python3 tools/pg_whatif.py

bench.py's PipelinedGraphStep at C3 timed in four forms over the same captured graphs:
  full      the benched step;
  no_geo    stream A only: the step graphs replayed, the geometry graphs not (every composite reuses
            the geometry its set already holds) -- the step without the other stream's contention;
  geo_only  stream B only: one geometry graph per step, back to back;
  serial    both, one after the other on one stream (no overlap).
full vs max(no_geo, geo_only) shows how much the two streams slow each other down.
"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from langsplat_amd.pipeline import PipelinedGraphStep
    from langsplat_amd.synthetic import CONFIGS, make_cameras, make_gaussians
    steps = int(os.environ.get("WI_STEPS", "300"))
    reps = int(os.environ.get("WI_REPS", "3"))
    c = CONFIGS[os.environ.get("WI_CONFIG", "C3")]
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
    real_geometry = pg._geometry
    sa, sb = pg.streams

    def timed(fn):
        out = []
        for _ in range(reps):
            time.sleep(0.02)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(steps):
                fn(k)
            pg.synchronize()
            torch.cuda.synchronize()
            out.append(1e3 * (time.perf_counter() - t0) / steps)
        return out

    def geo_only(k):
        with torch.cuda.stream(sb):
            pg.g_geo[k % pg.S].replay()

    def serial(k):
        p = k % pg.S
        with torch.cuda.stream(sa):
            pg.g_geo[p].replay()
            pg.g_comp[p].replay()

    forms = [("full", lambda k: pg.replay()), ("geo_only", geo_only), ("serial", serial)]
    for name, fn in forms:
        r = timed(fn)
        print(f"{name:9s} " + " ".join(f"{x:.4f}" for x in r) + f"  median {statistics.median(r):.4f} ms/step",
              flush=True)
    pg._geometry = lambda *a, **kw: None
    r = timed(lambda k: pg.replay())
    print(f"{'no_geo':9s} " + " ".join(f"{x:.4f}" for x in r) + f"  median {statistics.median(r):.4f} ms/step",
          flush=True)
    pg._geometry = real_geometry


if __name__ == "__main__":
    main()
