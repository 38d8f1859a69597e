"""langsplat_amd -- MI355X-native differentiable Gaussian rasterizer for LangSplat.

The hot path (forward + backward of RasterizeGaussians, BASELINE.json north_star) is
implemented as HIP kernels for gfx950 in csrc/, exposed through the C ABI of include/lsr.h
(liblsr.so) and wrapped here with the reference's Python API.
"""
from .rasterizer import GaussianRasterizationSettings, GaussianRasterizer, rasterize_gaussians  # noqa: F401

__all__ = ["GaussianRasterizationSettings", "GaussianRasterizer", "rasterize_gaussians"]
