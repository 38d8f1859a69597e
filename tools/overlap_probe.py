"""Probe: how much of the next view's forward hides behind this view's render backward (measurement
aid, C3 language step without the optimizer).

    python tools/overlap_probe.py [steps]

serial:     forward(k) + backward(k), one stream.
pipelined:  backward(k) on the main stream while forward(k + 1) runs on a side stream (geometry is
            frozen in the language step, so the next forward does not depend on this backward).
Views alternate between two streams; every step's autograd graph is kept alive to the end (no
buffer reuse across the streams).
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from langsplat_amd.synthetic import CONFIGS, make_cameras, make_gaussians  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    c = CONFIGS["C3"]
    P, W, H = c["P"], c["width"], c["height"]
    dev = torch.device("cuda", 0)
    model = bench.Model(make_gaussians(P, seed=0).to(dev), include_feature=True)
    cam = make_cameras(1, W, H, device=dev)[0]
    bg = torch.zeros(3, device=dev)
    gen = torch.Generator().manual_seed(100)
    gt = torch.nn.functional.normalize(torch.randn((3, H, W), generator=gen), dim=0).to(dev)
    mask = (torch.rand((1, H, W), generator=gen) < 0.9).to(dev)

    def fwd():
        return bench.render(cam, model, bench.Pipe, bg, bench.Opt, language_target=(gt, mask))["language_l1"]

    keep = []
    for _ in range(3):
        loss = fwd()
        loss.backward()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = fwd()
        loss.backward()
        keep.append(loss)
    torch.cuda.synchronize()
    serial = (time.perf_counter() - t0) / steps
    model._language_feature.grad = None

    # autograd runs a node's backward on its forward's stream: views alternate between two streams,
    # so backward(k) (stream k % 2) overlaps forward(k + 1) (the other stream)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for s in streams:
        s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(streams[0]):
        loss = fwd()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        cur = loss
        cur.backward()
        with torch.cuda.stream(streams[(k + 1) % 2]):
            loss = fwd()
        keep.append(cur)
        model._language_feature.grad = None
    torch.cuda.synchronize()
    piped = (time.perf_counter() - t0) / steps
    print(f"serial {serial * 1e3:.4f} ms/step, pipelined {piped * 1e3:.4f} ms/step")


if __name__ == "__main__":
    main()
