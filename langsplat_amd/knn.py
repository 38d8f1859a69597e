"""distCUDA2 on the GPU.

`from simple_knn._C import distCUDA2` (scene/gaussian_model.py:20) initialises the Gaussian scales
from the SfM point cloud (:180): for every point, the mean squared distance to its 3 nearest other
points.  Here it is liblsr.so's lsr_dist_cuda2 (exact grid search, langsplat_amd/csrc/lsr_knn.hip);
the `simple_knn` package in this repository re-exports it under the reference's import path.
"""
from __future__ import annotations

import ctypes

import torch

from . import _native


def dist_cuda2(points: torch.Tensor) -> torch.Tensor:
    """(N, 3) float points on a ROCm device -> (N,) float32 mean squared 3-NN distances."""
    if points.device.type != "cuda":
        raise RuntimeError("distCUDA2: points must be on a ROCm GPU device; there is no CPU path")
    if points.dim() != 2 or points.shape[1] != 3:
        raise ValueError(f"distCUDA2: expected (N, 3) points, got {tuple(points.shape)}")
    pts = points.detach().to(torch.float32).contiguous()
    N = pts.shape[0]
    out = torch.empty((N,), dtype=torch.float32, device=pts.device)
    if N == 0:
        return out
    alloc = _native._Allocator(pts.device)
    with _native._on_device(pts.device), alloc:
        _native._check(_native.load().lsr_dist_cuda2(N, ctypes.c_void_p(pts.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                                     _native._ALLOC_CB, None, _native._stream(pts.device)),
                       "lsr_dist_cuda2")
    return out
