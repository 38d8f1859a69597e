"""Small seeded scenes shared by the CPU and GPU tests (SURVEY.md §8d generators, reduced)."""
import math
from types import SimpleNamespace

import torch

from langsplat_amd.synthetic import activated_inputs, make_cameras, make_gaussians


def settings_for(cam, sh_degree=3, bg=(0.0, 0.0, 0.0), include_feature=True, scale_modifier=1.0,
                 device="cpu", debug=False, prefiltered=False):
    from langsplat_amd.rasterizer import GaussianRasterizationSettings
    cam = cam.to(device)
    return GaussianRasterizationSettings(
        image_height=int(cam.image_height), image_width=int(cam.image_width),
        tanfovx=math.tan(cam.FoVx * 0.5), tanfovy=math.tan(cam.FoVy * 0.5),
        bg=torch.tensor(bg, dtype=torch.float32, device=device), scale_modifier=scale_modifier,
        viewmatrix=cam.world_view_transform, projmatrix=cam.full_proj_transform, sh_degree=sh_degree,
        campos=cam.camera_center, prefiltered=prefiltered, debug=debug, include_feature=include_feature)


def scene(P=300, W=64, H=48, seed=0, view=0, n_views=1, sh_degree=3, extent=1.0, scale_range=(0.02, 0.12),
          include_feature=True, bg=(0.0, 0.0, 0.0), scale_modifier=1.0):
    """Returns (settings (CPU tensors), inputs dict of activated CPU float32 tensors)."""
    g = make_gaussians(P, seed=seed, sh_degree=sh_degree, extent=extent, scale_range=scale_range)
    cams = make_cameras(n_views, W, H)
    st = settings_for(cams[view], sh_degree=sh_degree, bg=bg, include_feature=include_feature,
                      scale_modifier=scale_modifier)
    with torch.no_grad():
        inp = activated_inputs(g, include_feature=include_feature)
    inp = {k: v.detach().clone().contiguous() for k, v in inp.items()}
    return st, inp


def to_device(settings, inputs, device):
    st = settings._replace(bg=settings.bg.to(device), viewmatrix=settings.viewmatrix.to(device),
                           projmatrix=settings.projmatrix.to(device), campos=settings.campos.to(device))
    return st, {k: v.to(device) for k, v in inputs.items()}


def grad_seed(H, W, seed=1, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn((3, H, W), generator=g) * scale, torch.randn((3, H, W), generator=g) * scale)
