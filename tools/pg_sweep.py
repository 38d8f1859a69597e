"""Times bench.py's pipelined graph step (langsplat_amd.pipeline.PipelinedGraphStep, C3) in several
configurations in one process (measurement aid):

    python3 tools/pg_sweep.py 2:start:1 3:start:1 3:fwd:1 2:start:0 [--steps 200]

each argument = buffer sets : geometry start ("start" with the step, "fwd" after the compositing) :
fused tail (1 = Adam inside the backward's epilogue, 0 = separate launches).  Every configuration is
timed twice, interleaved, on the same model (its language feature keeps training)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from langsplat_amd.pipeline import PipelinedGraphStep
    from langsplat_amd.synthetic import CONFIGS, make_cameras, make_gaussians
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 200
    args = [a for a in args if not a.isdigit()]
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
    fwd = lambda: bench.render(cam, model, bench.Pipe, bg, bench.Opt, language_target=(gt, mask))["language_l1"]  # noqa: E731
    forms = {}
    for a in args:
        sets, geo, fused = a.split(":")
        os.environ["LSR_PG_GEO"] = geo
        os.environ["LSR_FUSED_TAIL"] = fused
        pg = PipelinedGraphStep(fwd, [model._language_feature], optim, sets=int(sets)).capture()
        forms[a] = pg
    res = {a: [] for a in args}
    for rnd in range(2):
        for a in args:
            pg = forms[a]
            for _ in range(10):
                pg.replay()
            pg.synchronize()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                pg.replay()
            pg.synchronize()
            torch.cuda.synchronize()
            res[a].append(1000.0 * (time.perf_counter() - t0) / steps)
            assert pg.check()
    for a in args:
        print(f"pg_sweep {a:12s} ms/step " + " ".join(f"{v:.4f}" for v in res[a]), flush=True)


if __name__ == "__main__":
    main()
