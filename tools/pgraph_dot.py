"""Dump the pipelined step's two captured graphs as DOT files (measurement aid):
    python tools/pgraph_dot.py  ->  gpurun_out/pgraph_{0,1}.dot
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from langsplat_amd.pipeline import PipelinedGraphStep  # noqa: E402
from langsplat_amd.synthetic import make_cameras, make_gaussians  # noqa: E402

_orig = torch.cuda.CUDAGraph


class _Dbg(_orig):
    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.enable_debug_mode()


def main():
    torch.cuda.CUDAGraph = _Dbg
    dev = torch.device("cuda", 0)
    P, W, H = 20000, 320, 240
    model = bench.Model(make_gaussians(P, seed=0).to(dev), include_feature=True)
    cam = make_cameras(1, W, H, device=dev)[0]
    bg = torch.zeros(3, device=dev)
    gt = torch.nn.functional.normalize(torch.randn((3, H, W)), dim=0).to(dev)
    mask = (torch.rand((1, H, W)) < 0.9).to(dev)
    optim = bench.AmdAdam([{"params": [model._language_feature], "lr": 0.0025}], lr=0.0, eps=1e-15)

    def fwd():
        return bench.render(cam, model, bench.Pipe, bg, bench.Opt, language_target=(gt, mask))["language_l1"]
    fwd().backward()
    optim.step()
    optim.zero_grad(set_to_none=True)
    pg = PipelinedGraphStep(fwd, [model._language_feature], optim).capture()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    for k in (0, 1):
        for name, g in (("geo", pg.g_geo[k]), ("comp", pg.g_comp[k]), ("step", pg.g_step[k])):
            if g is not None:  # no separate step graph when the composite and step are merged
                g.debug_dump(os.path.join(ROOT, "gpurun_out", f"pgraph_{name}_{k}.dot"))


if __name__ == "__main__":
    main()
