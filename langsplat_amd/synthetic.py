"""Synthetic Gaussian scenes and cameras for parity tests and benchmarks.

There is no network and no dataset: scenes are seeded random Gaussians of the shape LangSplat
trains (GaussianModel parameters, scene/gaussian_model.py:44-57 and :165-187), generated on the
CPU with torch.Generator so every path (HIP, oracle) sees identical bits.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List

import numpy as np
import torch

from .camera import Camera, focal2fov, fov2focal, look_at_origin, make_camera

# BASELINE.json "configs"
CONFIGS = {
    "C1": dict(P=10_000, width=400, height=300, views=1, sh_degree=3),
    "C2": dict(P=500_000, width=1280, height=720, views=1, sh_degree=3),
    "C3": dict(P=1_000_000, width=1920, height=1080, views=1, sh_degree=3),
    "C4": dict(P=1_000_000, width=1920, height=1080, views=8, sh_degree=3),
    "C5": dict(P=3_000_000, width=1920, height=1080, views=8, sh_degree=3),
}


@dataclass
class GaussianParams:
    """Raw (pre-activation) parameters, named as in GaussianModel."""
    xyz: torch.Tensor            # (P, 3)
    features_dc: torch.Tensor    # (P, 1, 3)
    features_rest: torch.Tensor  # (P, K-1, 3)
    scaling: torch.Tensor        # (P, 3)  log scale
    rotation: torch.Tensor       # (P, 4)  unnormalised quaternion
    opacity: torch.Tensor        # (P, 1)  logit
    language_feature: torch.Tensor  # (P, 3) unnormalised
    max_sh_degree: int = 3

    @property
    def P(self) -> int:
        return self.xyz.shape[0]

    def to(self, device) -> "GaussianParams":
        return GaussianParams(*(getattr(self, f).to(device) for f in (
            "xyz", "features_dc", "features_rest", "scaling", "rotation", "opacity", "language_feature")),
            max_sh_degree=self.max_sh_degree)

    def tensors(self):
        return [self.xyz, self.features_dc, self.features_rest, self.scaling, self.rotation, self.opacity,
                self.language_feature]


def make_gaussians(P: int, seed: int = 0, sh_degree: int = 3, extent: float = 1.0,
                   scale_range=(0.003, 0.03)) -> GaussianParams:
    g = torch.Generator().manual_seed(seed)
    K = (sh_degree + 1) ** 2
    xyz = (torch.rand((P, 3), generator=g) * 2.0 - 1.0) * extent
    lo, hi = math.log(scale_range[0]), math.log(scale_range[1])
    scaling = torch.rand((P, 3), generator=g) * (hi - lo) + lo
    rotation = torch.randn((P, 4), generator=g)
    opacity = torch.randn((P, 1), generator=g) * 1.5
    f_dc = torch.randn((P, 1, 3), generator=g) * 0.5
    f_rest = torch.randn((P, K - 1, 3), generator=g) * 0.05
    lang = torch.randn((P, 3), generator=g)
    return GaussianParams(xyz, f_dc, f_rest, scaling, rotation, opacity, lang, sh_degree)


def make_cameras(n_views: int, width: int, height: int, radius: float = 4.0, fovy_deg: float = 50.0,
                 device="cpu") -> List[Camera]:
    """View 0 sits at (0, 0, -radius) looking +z; n views lie on a circle around the origin."""
    fovy = math.radians(fovy_deg)
    fovx = focal2fov(fov2focal(fovy, height), width)
    cams = []
    for k in range(n_views):
        th = 2.0 * math.pi * k / max(n_views, 1)
        pos = np.array([radius * math.sin(th), 0.0, -radius * math.cos(th)])
        R, T = look_at_origin(pos)
        cams.append(make_camera(R, T, fovx, fovy, width, height, device=device))
    return cams


def activated_inputs(params: GaussianParams, include_feature: bool = True):
    """The activated rasterizer inputs of gaussian_renderer/__init__.py:55-91 (differentiable)."""
    xyz = params.xyz
    opacity = torch.sigmoid(params.opacity)
    scales = torch.exp(params.scaling)
    rotations = torch.nn.functional.normalize(params.rotation)
    shs = torch.cat((params.features_dc, params.features_rest), dim=1)
    if include_feature:
        lf = params.language_feature
        lang = lf / (lf.norm(dim=-1, keepdim=True) + 1e-9)
    else:
        lang = torch.zeros((1,), dtype=opacity.dtype, device=opacity.device)
    return dict(means3D=xyz, opacities=opacity, scales=scales, rotations=rotations, shs=shs,
                language_feature_precomp=lang)
