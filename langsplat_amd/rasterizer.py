"""GaussianRasterizationSettings / GaussianRasterizer -- the reference's rasterizer API on MI355X.

Drop-in for `from diff_gaussian_rasterization import GaussianRasterizationSettings,
GaussianRasterizer` (gaussian_renderer/__init__.py:15).  Construction mirrors
gaussian_renderer/__init__.py:37-53, the call mirrors :96-105 and the return value is the
3-tuple unpacked there: (rendered_image (3,H,W), language_feature_image (3,H,W), radii (P,)).

Gradient semantics: `means2D` is a value-ignored sink whose .grad receives
dL/d(screen-space mean) in columns 0-1; gradients for opacities / scales / rotations /
language_feature_precomp are w.r.t. the activated tensors the caller passes in.

All work runs in liblsr.so (HIP kernels for gfx950) through the C ABI; CPU tensors are
rejected -- there is deliberately no CPU path here.
"""
from __future__ import annotations

from typing import NamedTuple

import torch
import torch.nn as nn

from . import _native


class GaussianRasterizationSettings(NamedTuple):
    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    bg: torch.Tensor
    scale_modifier: float
    viewmatrix: torch.Tensor
    projmatrix: torch.Tensor
    sh_degree: int
    campos: torch.Tensor
    prefiltered: bool
    debug: bool
    include_feature: bool = False


def _f32(t):
    if t is None or t.numel() == 0:
        return t
    if t.dtype != torch.float32:
        t = t.to(torch.float32)
    return t if t.is_contiguous() else t.contiguous()


def _cpu_deep_copy(args):
    return tuple(a.detach().cpu().clone() if isinstance(a, torch.Tensor) else a for a in args)


def rasterize_gaussians(means3D, means2D, sh, colors_precomp, language_feature_precomp, opacities, scales,
                        rotations, cov3Ds_precomp, raster_settings):
    return _RasterizeGaussians.apply(means3D, means2D, sh, colors_precomp, language_feature_precomp, opacities,
                                     scales, rotations, cov3Ds_precomp, raster_settings)


class _RasterizeGaussians(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means3D, means2D, sh, colors_precomp, language_feature_precomp, opacities, scales, rotations,
                cov3Ds_precomp, raster_settings):
        if means3D.device.type != "cuda":
            raise RuntimeError("langsplat_amd rasterizer: inputs must be on a ROCm GPU device "
                               f"(got {means3D.device}); there is no CPU implementation")
        P = means3D.shape[0]
        lang = language_feature_precomp
        use_lang = bool(raster_settings.include_feature) and lang is not None and lang.numel() == 3 * P and P > 0
        lang_in = _f32(lang) if use_lang else None
        args = (_f32(means3D), _f32(sh), _f32(colors_precomp), lang_in, _f32(opacities), _f32(scales),
                _f32(rotations), _f32(cov3Ds_precomp))
        if raster_settings.debug:
            cpu_args = _cpu_deep_copy(args)
            try:
                out = _native.rasterize_gaussians(raster_settings, *args)
            except Exception as ex:
                torch.save(cpu_args, "snapshot_fw.dump")
                print("\nAn error occured in forward. Please forward snapshot_fw.dump for debugging.")
                raise ex
        else:
            out = _native.rasterize_gaussians(raster_settings, *args)
        num_rendered, color, language_feature, radii, geom, binning, image = out
        ctx.raster_settings = raster_settings
        ctx.num_rendered = num_rendered
        ctx.use_lang = use_lang
        m3, shs_, cp, ln, op, sc, ro, cv = args
        ctx.save_for_backward(m3, shs_, cp, ln if ln is not None else torch.empty(0), sc, ro, cv, radii, geom,
                              binning, image)
        ctx.mark_non_differentiable(radii)
        return color, language_feature, radii

    @staticmethod
    def backward(ctx, grad_out_color, grad_out_language_feature, _grad_radii):
        rs = ctx.raster_settings
        means3D, sh, colors_precomp, lang, scales, rotations, cov3Ds_precomp, radii, geom, binning, image = \
            ctx.saved_tensors
        if grad_out_color is None:
            grad_out_color = torch.zeros((3, rs.image_height, rs.image_width), device=means3D.device)
        gl = grad_out_language_feature if ctx.use_lang else None
        args = (means3D, sh, colors_precomp, lang if ctx.use_lang else None, scales, rotations, cov3Ds_precomp,
                radii, grad_out_color, gl, ctx.num_rendered, geom, binning, image)
        if rs.debug:
            cpu_args = _cpu_deep_copy(args)
            try:
                g = _native.rasterize_gaussians_backward(rs, *args)
            except Exception as ex:
                torch.save(cpu_args, "snapshot_bw.dump")
                print("\nAn error occured in backward. Writing snapshot_bw.dump for debugging.\n")
                raise ex
        else:
            g = _native.rasterize_gaussians_backward(rs, *args)

        def want(i, t):
            return t if ctx.needs_input_grad[i] else None

        return (want(0, g["means3D"]), want(1, g["means2D"]), want(2, g["shs"]), want(3, g["colors_precomp"]),
                want(4, g["language_feature_precomp"] if ctx.use_lang else None), want(5, g["opacities"]),
                want(6, g["scales"]), want(7, g["rotations"]), want(8, g["cov3D_precomp"]), None)


class GaussianRasterizer(nn.Module):
    def __init__(self, raster_settings):
        super().__init__()
        self.raster_settings = raster_settings

    def markVisible(self, positions):
        # Mark visible points (based on frustum culling for camera) with a boolean
        with torch.no_grad():
            rs = self.raster_settings
            visible = _native.mark_visible(positions, rs.viewmatrix, rs.projmatrix)
        return visible

    def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, language_feature_precomp=None,
                scales=None, rotations=None, cov3D_precomp=None):
        raster_settings = self.raster_settings

        if (shs is None and colors_precomp is None) or (shs is not None and colors_precomp is not None):
            raise Exception('Please provide excatly one of either SHs or precomputed colors!')

        if ((scales is None or rotations is None) and cov3D_precomp is None) or \
                ((scales is not None or rotations is not None) and cov3D_precomp is not None):
            raise Exception('Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!')

        empty = torch.Tensor([])
        if shs is None:
            shs = empty
        if colors_precomp is None:
            colors_precomp = empty
        if language_feature_precomp is None:
            language_feature_precomp = empty
        if scales is None:
            scales = empty
        if rotations is None:
            rotations = empty
        if cov3D_precomp is None:
            cov3D_precomp = empty

        # Invoke the MI355X rasterization routine
        return rasterize_gaussians(means3D, means2D, shs, colors_precomp, language_feature_precomp, opacities,
                                   scales, rotations, cov3D_precomp, raster_settings)
