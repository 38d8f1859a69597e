"""Lane-utilisation statistics of the render backward at a BASELINE config (measurement aid).

    LSR_RENDER_STATS=1 python tools/render_stats.py [C3]
"""
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("LSR_RENDER_STATS", "1")

from langsplat_amd import _native  # noqa: E402
from langsplat_amd.rasterizer import GaussianRasterizationSettings  # noqa: E402
from langsplat_amd.synthetic import CONFIGS, activated_inputs, make_cameras, make_gaussians  # noqa: E402


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
        st, inp["means3D"], inp["shs"], None, inp["language_feature_precomp"], inp["opacities"], inp["scales"],
        inp["rotations"], None)
    _native.debug_render_stats()  # clear
    gc = torch.randn((3, H, W), device=dev) / (3 * H * W)
    gl = torch.randn((3, H, W), device=dev) / (3 * H * W)
    _native.rasterize_gaussians_backward(st, inp["means3D"], inp["shs"], None, inp["language_feature_precomp"],
                                         inp["scales"], inp["rotations"], None, radii, gc, gl, nr, geom, binning,
                                         image)
    torch.cuda.synchronize()
    s = _native.debug_render_stats()
    e, ph, ah, lh = s["entries"], s["power_hit"], s["alpha_hit"], s["lanes_hit"]
    print(f"{cfg}: R={nr} wave-entries={e} power-hit={ph} ({ph / max(e, 1):.3f}) alpha-hit={ah} "
          f"({ah / max(e, 1):.3f}) lanes/alpha-hit={lh / max(ah, 1):.2f} blends={lh}")
    print(f"  batches={s['batches']} wave-entry slots held by batch barriers (4 x busiest wave)="
          f"{s['barrier_slots']} -> wave utilisation {e / max(s['barrier_slots'], 1):.3f}")
    hist = s["hist"]
    tot = sum(hist)
    acc = 0
    for lo, hi in ((0, 0), (1, 2), (3, 4), (5, 8), (9, 16), (17, 32), (33, 64)):
        n = sum(hist[lo:hi + 1])
        acc += n
        print(f"  lanes {lo:2d}-{hi:2d}: {n / max(tot, 1):.3f} (cum {acc / max(tot, 1):.3f})")


if __name__ == "__main__":
    main()
