"""The language-feature loss around the rasterizer, on the GPU.

LangSplat's include_feature step (train.py:96-99) is

    gt, mask = viewpoint_cam.get_language_feature(language_feature_dir=..., feature_level=...)
    Ll1 = l1_loss(language_feature * mask, gt * mask)       # utils/loss_utils.py:17-18

`get_language_feature` (scene/cameras.py:58-92) np.loads two arrays, gathers on the CPU and
copies to the GPU every step; the loss is ~11 torch kernels forward + backward.  Here:

    cache = LanguageFeatureCache(device)
    gt, mask = cache.get(viewpoint_cam, dataset.lf_path, dataset.feature_level)   # decoded once, in HBM
    Ll1 = masked_l1_loss(language_feature, gt, mask)                                # 1 kernel each way

`masked_l1_loss(pred, gt, mask)` equals `l1_loss(pred * mask, gt * mask)` (same value up to
summation order; the gradient is bit-identical to torch autograd's).  All work runs in liblsr.so.
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, Tuple

import numpy as np
import torch

from . import _native


def _stream_ptr(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


_SCRATCH: Dict[Tuple[int, int], torch.Tensor] = {}


def _scratch(device: torch.device) -> torch.Tensor:
    """Per (device, stream) zero-initialised reduction scratch; the kernel leaves it zeroed."""
    key = (device.index if device.index is not None else torch.cuda.current_device(),
           torch.cuda.current_stream(device).cuda_stream)
    t = _SCRATCH.get(key)
    if t is None:
        nbytes = int(_native.load().lsr_masked_l1_scratch_bytes(3, 1))
        t = torch.zeros((nbytes,), dtype=torch.uint8, device=device)
        _SCRATCH[key] = t
    return t


def _mask_arg(mask: torch.Tensor, HW: int):
    if mask.numel() != HW:
        raise ValueError(f"mask must have H*W = {HW} elements (shape (1,H,W) or (H,W)), got {tuple(mask.shape)}")
    if mask.dtype == torch.bool or mask.dtype == torch.uint8:
        m = mask.contiguous().view(torch.uint8)
        return m, 0
    m = mask.to(torch.float32).contiguous()
    return m, 1


class _MaskedL1(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, gt, mask):
        if pred.device.type != "cuda":
            raise RuntimeError("masked_l1_loss: tensors must be on a ROCm GPU device; there is no CPU path")
        if pred.shape != gt.shape or pred.dim() != 3:
            raise ValueError(f"masked_l1_loss: pred and gt must both be (C,H,W); got {tuple(pred.shape)} and "
                             f"{tuple(gt.shape)}")
        C, H, W = pred.shape
        HW = H * W
        p = pred.detach().to(torch.float32).contiguous()
        g = gt.detach().to(torch.float32).contiguous()
        m, is_float = _mask_arg(mask, HW)
        loss = torch.empty((), dtype=torch.float32, device=pred.device)
        lib = _native.load()
        with _native._on_device(pred.device):
            _native._check(lib.lsr_masked_l1_forward(C, HW, _native._ptr(p), _native._ptr(g), _native._ptr(m), is_float,
                                                     ctypes.c_void_p(loss.data_ptr()),
                                                     ctypes.c_void_p(_scratch(pred.device).data_ptr()),
                                                     _stream_ptr(pred.device)), "lsr_masked_l1_forward")
        ctx.save_for_backward(p, g, m)
        ctx.is_float = is_float
        return loss

    @staticmethod
    def backward(ctx, grad_loss):
        p, g, m = ctx.saved_tensors
        C, H, W = p.shape
        gl = grad_loss.detach().to(torch.float32).contiguous()
        out = torch.empty_like(p)
        lib = _native.load()
        with _native._on_device(p.device):
            _native._check(lib.lsr_masked_l1_backward(C, H * W, _native._ptr(p), _native._ptr(g), _native._ptr(m),
                                                      ctx.is_float, ctypes.c_void_p(gl.data_ptr()), _native._ptr(out),
                                                      _stream_ptr(p.device)), "lsr_masked_l1_backward")
        return out, None, None


def masked_l1_loss(pred: torch.Tensor, gt: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    """l1_loss(pred * mask, gt * mask) of train.py:98 as one HIP kernel (backward: one more).
    pred, gt: (C,H,W) fp32 on the GPU; mask: (1,H,W) or (H,W), bool or float, broadcast over C."""
    return _MaskedL1.apply(pred, gt, mask)


def decode_language_feature(seg_map: torch.Tensor, feature_map: torch.Tensor, feature_level: int):
    """Camera.get_language_feature's gather (scene/cameras.py:63-92) on the GPU.

    seg_map: (L,H,W) segment ids (-1 = no segment), feature_map: (N,D).  Returns
    (feature (D,H,W) fp32, mask (1,H,W) bool) exactly as the reference builds them, including
    torch's reading of index -1 as the last feature row.  A segment id outside [-N, N) raises
    IndexError, as the reference's feature_map[seg] does."""
    if seg_map.dim() != 3:
        raise ValueError("seg_map must be (L,H,W)")
    L, H, W = seg_map.shape
    if not 0 <= int(feature_level) < L:
        raise ValueError("feature_level=", feature_level)
    device = feature_map.device
    seg = seg_map.to(device=device, dtype=torch.int64).contiguous()
    fm = feature_map.to(torch.float32).contiguous()
    N, D = fm.shape
    out = torch.empty((D, H, W), dtype=torch.float32, device=device)
    mask = torch.empty((1, H, W), dtype=torch.bool, device=device)
    lib = _native.load()
    with _native._on_device(device):
        status = lib.lsr_decode_language_feature(L, H, W, _native._ptr(seg), int(feature_level), N, D,
                                                 _native._ptr(fm), _native._ptr(out),
                                                 ctypes.c_void_p(mask.data_ptr()), _stream_ptr(device))
    if status == 1:  # LSR_ERR_INVALID: a segment id outside the feature map
        raise IndexError(f"decode_language_feature: {_native.last_error()}")
    _native._check(status, "lsr_decode_language_feature")
    return out, mask


class LanguageFeatureCache:
    """Per-view decoded ground truth kept in HBM (the reference reloads it from disk every step).

    A 1080p view costs 3*H*W*4 + H*W bytes (~27 MB), so even hundreds of views fit in 288 GB."""

    def __init__(self, device="cuda"):
        self.device = torch.device(device)
        self._maps: Dict[Tuple[str, str, int], Tuple[torch.Tensor, torch.Tensor]] = {}

    def get(self, camera, language_feature_dir: str, feature_level: int):
        key = (language_feature_dir, camera.image_name, int(feature_level))
        hit = self._maps.get(key)
        if hit is None:
            base = os.path.join(language_feature_dir, camera.image_name)
            seg = torch.from_numpy(np.load(base + "_s.npy"))           # allow_pickle=False (default)
            feat = torch.from_numpy(np.load(base + "_f.npy"))
            H, W = int(camera.image_height), int(camera.image_width)
            # scene/cameras.py:69-73 reads seg_map[:, y, x] for y < H, x < W: a larger map is cropped
            # to its top-left H x W, a smaller one raises IndexError there
            if seg.dim() != 3 or seg.shape[1] < H or seg.shape[2] < W:
                raise IndexError(f"{base}_s.npy is {tuple(seg.shape)}, smaller than the camera's {H}x{W}")
            seg = seg[:, :H, :W]
            hit = decode_language_feature(seg.to(self.device), feat.to(self.device), feature_level)
            self._maps[key] = hit
        return hit

    def __len__(self):
        return len(self._maps)
