"""Host enqueue time vs device time of the pipelined graph step at C3 (measurement aid):

    python3 tools/pg_host.py [--steps 300] [--nowait | --sync]

Prints the host time per replay() call (enqueue only) and the wall time per step to the final
synchronize: when they are close the host, not the GPU, sets the step rate.
"""
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
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 300
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
    wait = "--nowait" not in sys.argv
    sync = "--sync" in sys.argv
    for _ in range(20):
        pg.replay(wait=wait)
    pg.synchronize()
    torch.cuda.synchronize()
    walls = []
    for rep in range(int(os.environ.get("PG_HOST_REPS", "3"))):
        t0 = time.perf_counter()
        for _ in range(steps):
            if sync:  # train.py:108: loss.item() after every step
                pg.replay().item()
            else:
                pg.replay(wait=wait)
        t1 = time.perf_counter()
        pg.synchronize()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"pg_host rep {rep}: host enqueue {1e3 * (t1 - t0) / steps:.4f} ms/replay, "
              f"wall {1e3 * (t2 - t0) / steps:.4f} ms/step (ended at {time.time():.3f})", flush=True)
        walls.append(1e3 * (t2 - t0) / steps)
    walls.sort()
    print(f"pg_host summary: min {walls[0]:.4f} median {walls[len(walls) // 2]:.4f} ms/step", flush=True)


if __name__ == "__main__":
    main()
