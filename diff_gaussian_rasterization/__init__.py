"""Drop-in module name for LangSplat (gaussian_renderer/__init__.py:15 imports
`from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer`).

Re-exports the MI355X-native implementation from langsplat_amd; there is no CUDA extension.
"""
from langsplat_amd.rasterizer import (  # noqa: F401
    GaussianRasterizationSettings,
    GaussianRasterizer,
    _RasterizeGaussians,
    rasterize_gaussians,
)

__all__ = ["GaussianRasterizationSettings", "GaussianRasterizer", "rasterize_gaussians"]
