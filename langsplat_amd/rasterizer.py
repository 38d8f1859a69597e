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
    # grad mode is read HERE: inside Function.forward it is always off, and ctx.needs_input_grad
    # reflects requires_grad only (True under torch.no_grad() for a parameter that requires grad)
    return _RasterizeGaussians.apply(means3D, means2D, sh, colors_precomp, language_feature_precomp, opacities,
                                     scales, rotations, cov3Ds_precomp, raster_settings, torch.is_grad_enabled())


def _forward_flags(ctx, grad_enabled: bool) -> int:
    """A backward will follow (grad mode on and an input needs a gradient): the compositing kernel
    clears its gradient records.  None will (inference, render.py:24-55 under torch.no_grad()):
    LSR_FWD_NO_BACKWARD, the kernel writes no backward state."""
    return _native.FWD_ZERO_GRAD_RECORDS if grad_enabled and any(ctx.needs_input_grad) else _native.FWD_NO_BACKWARD


class _RasterizeGaussians(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means3D, means2D, sh, colors_precomp, language_feature_precomp, opacities, scales, rotations,
                cov3Ds_precomp, raster_settings, grad_enabled=True):
        if means3D.device.type != "cuda":
            raise RuntimeError("langsplat_amd rasterizer: inputs must be on a ROCm GPU device "
                               f"(got {means3D.device}); there is no CPU implementation")
        P = means3D.shape[0]
        lang = language_feature_precomp
        use_lang = bool(raster_settings.include_feature) and lang is not None and lang.numel() == 3 * P and P > 0
        lang_in = _f32(lang) if use_lang else None
        args = (_f32(means3D), _f32(sh), _f32(colors_precomp), lang_in, _f32(opacities), _f32(scales),
                _f32(rotations), _f32(cov3Ds_precomp))
        flags = _forward_flags(ctx, grad_enabled)
        ctx.records_zeroed = flags == _native.FWD_ZERO_GRAD_RECORDS
        if raster_settings.debug:
            cpu_args = _cpu_deep_copy(args)
            try:
                out = _native.rasterize_gaussians(raster_settings, *args, flags=flags)
            except Exception as ex:
                torch.save(cpu_args, "snapshot_fw.dump")
                print("\nAn error occured in forward. Please forward snapshot_fw.dump for debugging.")
                raise ex
        else:
            out = _native.rasterize_gaussians(raster_settings, *args, flags=flags)
        num_rendered, color, language_feature, radii, geom, binning, image = out
        ctx.raster_settings = raster_settings
        ctx.num_rendered = num_rendered
        ctx.use_lang = use_lang
        m3, shs_, cp, ln, op, sc, ro, cv = args
        ctx.save_for_backward(m3, shs_, cp, ln if ln is not None else torch.empty(0), sc, ro, cv, radii, geom,
                              binning, image)
        ctx.mark_non_differentiable(radii)
        ctx.set_materialize_grads(False)  # an output off the loss path arrives as None (= zeros)
        return color, language_feature, radii

    @staticmethod
    def backward(ctx, grad_out_color, grad_out_language_feature, _grad_radii):
        rs = ctx.raster_settings
        means3D, sh, colors_precomp, lang, scales, rotations, cov3Ds_precomp, radii, geom, binning, image = \
            ctx.saved_tensors
        gl = grad_out_language_feature if ctx.use_lang else None  # grad_out_color None: zero colour gradient
        args = (means3D, sh, colors_precomp, lang if ctx.use_lang else None, scales, rotations, cov3Ds_precomp,
                radii, grad_out_color, gl, ctx.num_rendered, geom, binning, image)
        geometry = _native.geometry_grads_needed(ctx.needs_input_grad, (0, 2, 3, 5, 6, 7, 8))
        flags = _native.BWD_RECORDS_ZEROED if ctx.records_zeroed else 0
        ctx.records_zeroed = False  # a second backward (retain_graph) clears its own records
        if rs.debug:
            cpu_args = _cpu_deep_copy(args)
            try:
                g = _native.rasterize_gaussians_backward(rs, *args, geometry=geometry, flags=flags)
            except Exception as ex:
                torch.save(cpu_args, "snapshot_bw.dump")
                print("\nAn error occured in backward. Writing snapshot_bw.dump for debugging.\n")
                raise ex
        else:
            g = _native.rasterize_gaussians_backward(rs, *args, geometry=geometry, flags=flags)

        def want(i, t):
            return t if ctx.needs_input_grad[i] else None

        return (want(0, g["means3D"]), want(1, g["means2D"]), want(2, g["shs"]), want(3, g["colors_precomp"]),
                want(4, g["language_feature_precomp"] if ctx.use_lang else None), want(5, g["opacities"]),
                want(6, g["scales"]), want(7, g["rotations"]), want(8, g["cov3D_precomp"]), None, None)


def rasterize_gaussians_fused(means3D, means2D, features_dc, features_rest, opacity_raw, scaling_raw, rotation_raw,
                              language_feature_raw, raster_settings, with_visibility=False, language_target=None):
    """Fused-activation form of the rasterizer call.

    Takes GaussianModel's RAW parameters -- _features_dc (P,1,3), _features_rest (P,M-1,3),
    _opacity (P,1), _scaling (P,3), _rotation (P,4), _language_feature (P,3) or None -- and
    returns exactly what GaussianRasterizer(...) returns for the activated inputs of
    gaussian_renderer/__init__.py:55-91: (color, language_feature_image, radii).  The kernels
    apply sigmoid / exp / normalize / the language normalisation and the SH concatenation
    themselves (include/lsr.h lsr_raw_flags), so those torch passes and their backward kernels
    disappear; gradients come back w.r.t. the raw parameters.  with_visibility=True appends
    render()'s visibility_filter (radii > 0, written by the preprocess kernel).

    language_target=(gt (3,H,W), mask (1,H,W) or (H,W) bool): also returns, last, LangSplat's
    language loss Ll1 = l1_loss(language_feature_image * mask, gt * mask) (train.py:96-99), computed
    by the compositing kernel from the pixels it produces; its backward is folded into the render
    backward's per-pixel seed (no separate loss kernels).
    """
    gt = mask = None
    if language_target is not None:
        gt, mask = language_target
        gt = _f32(gt.detach())
        mask = mask.detach()
        if mask.dtype != torch.bool:
            mask = mask != 0
        mask = mask.contiguous()
    color, lang, radii, visible, loss = _RasterizeGaussiansFused.apply(
        means3D, means2D, features_dc, features_rest, opacity_raw, scaling_raw, rotation_raw, language_feature_raw,
        raster_settings, gt, mask, torch.is_grad_enabled())
    out = (color, lang, radii, visible) if with_visibility else (color, lang, radii)
    return out + (loss,) if language_target is not None else out


def _guarded(rs, dump, msg, fn, args):
    """Run a native call; with debug=True snapshot its inputs and dump them on failure (upstream)."""
    if not rs.debug:
        return fn(*args)
    cpu_args = _cpu_deep_copy(args)
    try:
        return fn(*args)
    except Exception as ex:
        torch.save(cpu_args, dump)
        print(msg)
        raise ex


class _RasterizeGaussiansFused(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means3D, means2D, features_dc, features_rest, opacity_raw, scaling_raw, rotation_raw,
                language_feature_raw, raster_settings, loss_target=None, loss_mask=None, grad_enabled=True):
        if means3D.device.type != "cuda":
            raise RuntimeError("langsplat_amd rasterizer: inputs must be on a ROCm GPU device "
                               f"(got {means3D.device}); there is no CPU implementation")
        P = means3D.shape[0]
        lang = language_feature_raw
        use_lang = bool(raster_settings.include_feature) and lang is not None and lang.numel() == 3 * P and P > 0
        raw = _native.RAW_OPACITY | _native.RAW_SCALES | _native.RAW_ROTATIONS | (
            _native.RAW_LANGUAGE if use_lang else 0)
        rest = _f32(features_rest) if features_rest is not None and features_rest.numel() > 0 else None
        m3, dc, ln, op, sc, ro = (_f32(means3D), _f32(features_dc), _f32(lang) if use_lang else None,
                                  _f32(opacity_raw), _f32(scaling_raw), _f32(rotation_raw))
        visible = _native.output_tensor("visible", (P,), torch.bool, m3.device)  # radii > 0, written by preprocess
        fuse_loss = loss_target is not None
        if fuse_loss and not raster_settings.include_feature:
            raise ValueError("the fused language loss needs include_feature=True")
        # without the fused loss this output is never handed to the caller (no fill kernel)
        loss = _native.output_tensor("loss", (), torch.float32, m3.device)
        flags = _forward_flags(ctx, grad_enabled)
        ctx.records_zeroed = flags == _native.FWD_ZERO_GRAD_RECORDS
        # the language step (train.py:96-104): the loss is the fused language loss, so the colour
        # image is expected off the loss path and the split-replay states skip the colour sums; a
        # colour gradient arriving anyway is served by rasterizing again with them (backward below)
        ctx.no_color = fuse_loss and ctx.records_zeroed
        if ctx.no_color:
            flags |= _native.FWD_NO_COLOR_GRAD
        # a pipelined step (the composite half of a split forward, or a forward deferring the feature
        # to another stream's update): another stream's kernels run beside this view's backward
        ctx.shared_cu = (_native.forward_phase.active() in (_native.forward_phase.COMPOSITE,
                                                            _native.forward_phase.COMPOSITE_FILLED)
                         or _native.language_ready.active() is not None)

        def run(fwd_flags, vis, out_loss):
            return _guarded(raster_settings, "snapshot_fw.dump",
                            "\nAn error occured in forward. Please forward snapshot_fw.dump for debugging.",
                            lambda *a: _native.rasterize_gaussians(raster_settings, *a[:8], raw=raw, shs_rest=a[8],
                                                                   visible=a[9], loss_target=a[10], loss_mask=a[11],
                                                                   out_loss=a[12], flags=fwd_flags),
                            (m3, dc, None, ln, op, sc, ro, None, rest, vis, loss_target, loss_mask,
                             out_loss if fuse_loss else None))
        out = run(flags, visible, loss)
        if ctx.no_color:
            dev = m3.device  # (the closure holds inputs only: an output in ctx would form a cycle)
            ctx.rerun = lambda: run(flags & ~_native.FWD_NO_COLOR_GRAD, torch.empty((P,), dtype=torch.bool, device=dev),
                                    torch.empty((), dtype=torch.float32, device=dev))
        num_rendered, color, language_feature, radii, geom, binning, image = out
        ctx.raster_settings = raster_settings
        ctx.num_rendered = num_rendered
        ctx.use_lang = use_lang
        ctx.raw = raw
        ctx.rest_shape = tuple(features_rest.shape) if features_rest is not None else None
        empty = torch.empty(0)
        ctx.save_for_backward(m3, dc, rest if rest is not None else empty, ln if ln is not None else empty, op, sc,
                              ro, radii, geom, binning, image)
        ctx.fuse_loss = fuse_loss
        ctx.mark_non_differentiable(radii, visible)
        if not fuse_loss:
            ctx.mark_non_differentiable(loss)
        ctx.set_materialize_grads(False)  # an output off the loss path arrives as None (= zeros)
        return color, language_feature, radii, visible, loss

    @staticmethod
    def backward(ctx, grad_out_color, grad_out_language_feature, _grad_radii, _grad_visible, grad_loss=None):
        rs = ctx.raster_settings
        m3, dc, rest, ln, op, sc, ro, radii, geom, binning, image = ctx.saved_tensors
        num_rendered = ctx.num_rendered
        if grad_out_color is not None and ctx.no_color:
            # the forward kept no colour sums (include/lsr.h LSR_FWD_NO_COLOR_GRAD): the same forward
            # again with them (bit-identical outputs), then the backward reads its buffers
            if (torch.cuda.is_current_stream_capturing() or _native.static_buffers.active() is not None
                    or _native.language_ready.active() is not None):
                raise RuntimeError("a colour gradient reached a rasterizer call made with language_target "
                                   "inside a captured or pipelined step; render with language_target=None and "
                                   "form the language loss as a torch op when the colour image is in the loss")
            num_rendered, _, _, _, geom, binning, image = ctx.rerun()
        rest = rest if rest.numel() > 0 else None  # grad_out_color None: zero colour gradient
        gl = grad_out_language_feature if ctx.use_lang else None
        geometry = _native.geometry_grads_needed(ctx.needs_input_grad, (0, 2, 3, 4, 5, 6))
        flags = (_native.BWD_RECORDS_ZEROED if ctx.records_zeroed else 0) | (
            _native.BWD_SHARED_CU if ctx.shared_cu else 0)
        ctx.records_zeroed = False  # a second backward (retain_graph) clears its own records
        # a captured N = 1 language step may fuse its Adam step into this backward's epilogue
        fu = _native.fused_update.active()
        if not (fu is not None and ctx.use_lang and not geometry and grad_out_color is None
                and ctx.needs_input_grad[7] and ln.numel() > 0 and ln.data_ptr() == fu.param.data_ptr()):
            fu = None
        g = _guarded(rs, "snapshot_bw.dump",
                     "\nAn error occured in backward. Writing snapshot_bw.dump for debugging.\n",
                     lambda *a: _native.rasterize_gaussians_backward(rs, *a[:14], raw=ctx.raw, shs_rest=a[14],
                                                                     opacities=a[15], geometry=geometry,
                                                                     grad_loss=a[16], flags=flags, update=fu),
                     (m3, dc, None, ln if ctx.use_lang else None, sc, ro, None, radii, grad_out_color, gl,
                      num_rendered, geom, binning, image, rest, op,
                      grad_loss if ctx.fuse_loss and ctx.use_lang else None))

        def want(i, t):
            return t if ctx.needs_input_grad[i] else None

        d_rest = g.get("shs_rest")
        if d_rest is None and ctx.rest_shape is not None and ctx.needs_input_grad[3]:
            d_rest = torch.zeros(ctx.rest_shape, dtype=torch.float32, device=m3.device)
        return (want(0, g["means3D"]), want(1, g["means2D"]), want(2, g["shs"]), want(3, d_rest),
                want(4, g["opacities"]), want(5, g["scales"]), want(6, g["rotations"]),
                want(7, g["language_feature_precomp"] if ctx.use_lang else None), None, None, None, None)


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
