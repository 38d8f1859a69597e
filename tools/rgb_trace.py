"""Kernel trace of bench.RGBStep (the RGB stage's step at C3; measurement aid):

    rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rgb -o t -- python3 tools/rgb_trace.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if __name__ == "__main__":
    import torch
    import bench
    from langsplat_amd.synthetic import CONFIGS, make_cameras, make_gaussians
    c = CONFIGS["C3"]
    dev = torch.device("cuda", 0)
    cam = make_cameras(1, c["width"], c["height"], device=dev)[0]
    gt = torch.rand((3, c["height"], c["width"]), generator=torch.Generator().manual_seed(200)).to(dev)
    step = bench.RGBStep(make_gaussians(c["P"], seed=0, sh_degree=c["sh_degree"]).to(dev), cam, gt)
    for _ in range(13):
        step()
    torch.cuda.synchronize()
