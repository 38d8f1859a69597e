"""Per-tile work distribution of the render kernels at a BASELINE config (measurement aid).

    python tools/tile_stats.py [C3]

Prints the list length and the backward's replay length (max n_contrib of the tile) per tile,
their percentiles, and the makespan of the tile -> workgroup-slot schedule the hardware runs
(tiles in launch order onto the first free slot) relative to perfect balance, for a few
workgroups-per-CU occupancies.
"""
import heapq
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from langsplat_amd import _native  # noqa: E402
from langsplat_amd.rasterizer import GaussianRasterizationSettings  # noqa: E402
from langsplat_amd.synthetic import CONFIGS, activated_inputs, make_cameras, make_gaussians  # noqa: E402


def makespan(work, slots):
    free = [0.0] * slots
    heapq.heapify(free)
    end = 0.0
    for w in work:
        t = heapq.heappop(free) + w
        end = max(end, t)
        heapq.heappush(free, t)
    return end


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
    c = CONFIGS[cfg]
    dev = torch.device("cuda")
    P, W, H = c["P"], c["width"], c["height"]
    g = make_gaussians(P, seed=0).to(dev)
    cam = make_cameras(1, W, H, device=dev)[0]
    st = GaussianRasterizationSettings(H, W, math.tan(cam.FoVx * 0.5), math.tan(cam.FoVy * 0.5),
                                       torch.zeros(3, device=dev), 1.0, cam.world_view_transform,
                                       cam.full_proj_transform, 3, cam.camera_center, False, False, True)
    with torch.no_grad():
        inp = activated_inputs(g)
        nr, color, lang, radii, geom, binning, image = _native.rasterize_gaussians(
            st, inp["means3D"], inp["shs"], None, inp["language_feature_precomp"], inp["opacities"],
            inp["scales"], inp["rotations"], None)
    lay = _native.state_layout(P, W, H, nr)
    gx, gy = (W + 15) // 16, (H + 15) // 16
    T = gx * gy
    rng = image[lay["ranges"]:lay["ranges"] + 8 * T].view(torch.int32).view(T, 2).cpu().numpy().astype(np.int64)
    length = rng[:, 1] - rng[:, 0]
    nc = image[lay["n_contrib"]:lay["n_contrib"] + 4 * W * H].view(torch.int32).cpu().numpy().reshape(H, W)
    pad = np.zeros((gy * 16, gx * 16), np.int64)
    pad[:H, :W] = nc
    maxl = pad.reshape(gy, 16, gx, 16).max(axis=(1, 3)).reshape(-1)
    print(f"{cfg}: tiles={T} nonempty={int((length > 0).sum())} replaying={int((maxl > 0).sum())} "
          f"R={nr} sum(maxl)={int(maxl.sum())}")
    for name, a in (("list length", length), ("replay length", maxl)):
        nz = a[a > 0]
        q = np.percentile(nz, [50, 90, 99, 100]) if nz.size else [0] * 4
        print(f"  {name:13s}: mean {nz.mean():.0f}  p50 {q[0]:.0f}  p90 {q[1]:.0f}  p99 {q[2]:.0f}  max {q[3]:.0f}")
    # the backward's per-tile time ~ a fixed cost + batches of 256 replayed entries
    work = maxl.astype(np.float64) + 64.0
    for per_cu in (4, 5, 6, 8):
        slots = 256 * per_cu
        ms = makespan(work, slots)
        print(f"  {per_cu} workgroups/CU: makespan / balanced = {ms / (work.sum() / slots):.3f}")


if __name__ == "__main__":
    main()
