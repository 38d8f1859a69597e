"""Host-side cost of the bench's language train step (measurement aid): cProfile of K steps and the
host wall time per step, split into the time spent waiting on the GPU (the counter hand-off inside
lsr_forward, synchronize) and the rest (Python, autograd, launches).

    python tools/host_profile.py [steps] [config]
"""
import cProfile
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from langsplat_amd.optim import Adam as AmdAdam  # noqa: E402
from langsplat_amd.render import render  # noqa: E402
from langsplat_amd.synthetic import CONFIGS, make_cameras, make_gaussians  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    dev = torch.device("cuda", 0)
    c = CONFIGS[sys.argv[2] if len(sys.argv) > 2 else "C3"]
    params = make_gaussians(c["P"], seed=0, sh_degree=c["sh_degree"]).to(dev)
    model = bench.Model(params, include_feature=True)
    cam = make_cameras(1, c["width"], c["height"], device=dev)[0]
    bg = torch.zeros(3, device=dev)
    gen = torch.Generator().manual_seed(100)
    gt = torch.nn.functional.normalize(torch.randn((3, c["height"], c["width"]), generator=gen), dim=0).to(dev)
    mask = (torch.rand((1, c["height"], c["width"]), generator=gen) < 0.9).to(dev)
    optim = AmdAdam([{"params": [model._language_feature], "lr": 0.0025, "name": "language_feature"}], lr=0.0,
                    eps=1e-15)

    def step():
        loss = render(cam, model, bench.Pipe, bg, bench.Opt, language_target=(gt, mask))["language_l1"]
        loss.backward()
        optim.step()
        optim.zero_grad(set_to_none=True)

    for _ in range(10):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    print(f"{steps} steps: {1e3 * (time.perf_counter() - t0) / steps:.4f} ms/step")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
