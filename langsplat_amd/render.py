"""render() glue -- mirror of gaussian_renderer/__init__.py:19-115 over langsplat_amd.

Kept API-identical (same arguments, same returned dict) so that LangSplat's train.py / render.py
can use it; the only change is that inputs come from any object exposing the GaussianModel
getters (get_xyz, get_opacity, get_scaling, get_rotation, get_features, get_language_feature,
get_covariance, active_sh_degree, max_sh_degree).
"""
from __future__ import annotations

import math
import os

import torch

from . import _native
from .rasterizer import GaussianRasterizationSettings, GaussianRasterizer, rasterize_gaussians_fused


def _fusable(pc, pipe, override_color, device) -> bool:
    """True when render()'s inputs are GaussianModel's default activations of raw tensors
    (scene/gaussian_model.py:33-41), so the kernels can activate them.
    LANGSPLAT_AMD_FUSED=0 forces the reference's unfused call."""
    if os.environ.get("LANGSPLAT_AMD_FUSED", "1") == "0" or device.type != "cuda":
        return False
    if override_color is not None or pipe.convert_SHs_python or pipe.compute_cov3D_python:
        return False
    if not all(isinstance(getattr(pc, n, None), torch.Tensor)
               for n in ("_features_dc", "_features_rest", "_opacity", "_scaling", "_rotation")):
        return False
    return (getattr(pc, "scaling_activation", None) is torch.exp
            and getattr(pc, "opacity_activation", None) is torch.sigmoid
            and getattr(pc, "rotation_activation", None) is torch.nn.functional.normalize)


def eval_sh(deg, sh, dirs):
    """utils/sh_utils.py:57-112 for deg <= 3 (used only by the convert_SHs_python switch)."""
    C0 = 0.28209479177387814
    C1 = 0.4886025119029199
    C2 = [1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396]
    C3 = [-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
          1.445305721320277, -0.5900435899266435]
    result = C0 * sh[..., 0]
    if deg > 0:
        x, y, z = dirs[..., 0:1], dirs[..., 1:2], dirs[..., 2:3]
        result = result - C1 * y * sh[..., 1] + C1 * z * sh[..., 2] - C1 * x * sh[..., 3]
        if deg > 1:
            xx, yy, zz = x * x, y * y, z * z
            xy, yz, xz = x * y, y * z, x * z
            result = (result + C2[0] * xy * sh[..., 4] + C2[1] * yz * sh[..., 5] +
                      C2[2] * (2.0 * zz - xx - yy) * sh[..., 6] + C2[3] * xz * sh[..., 7] +
                      C2[4] * (xx - yy) * sh[..., 8])
            if deg > 2:
                result = (result + C3[0] * y * (3 * xx - yy) * sh[..., 9] + C3[1] * xy * z * sh[..., 10] +
                          C3[2] * y * (4 * zz - xx - yy) * sh[..., 11] +
                          C3[3] * z * (2 * zz - 3 * xx - 3 * yy) * sh[..., 12] +
                          C3[4] * x * (4 * zz - xx - yy) * sh[..., 13] + C3[5] * z * (xx - yy) * sh[..., 14] +
                          C3[6] * x * (xx - 3 * yy) * sh[..., 15])
    return result


_ZEROS: dict = {}


def _screenspace_points(xyz: torch.Tensor) -> torch.Tensor:
    """viewspace_points of gaussian_renderer/__init__.py:24-28: a zero (P,3) tensor that requires
    grad and whose .grad receives dL/dmeans2D after backward.

    The reference builds `zeros_like(xyz, requires_grad=True) + 0` and retain_grad()s it: per step
    a fill, an add, and a clone of the incoming gradient.  Here it is a fresh leaf over a cached
    zero buffer.  It has the same values and the same .grad, and autograd hands the rasterizer's
    gradient to .grad without a copy."""
    key = (xyz.device, xyz.dtype, int(xyz.shape[0]))
    z = _ZEROS.get(key)
    if z is None:
        _ZEROS.clear()
        z = torch.zeros((int(xyz.shape[0]), 3), dtype=xyz.dtype, device=xyz.device)
        _ZEROS[key] = z
    return z.detach().requires_grad_(True)


def render(viewpoint_camera, pc, pipe, bg_color: torch.Tensor, opt, scaling_modifier=1.0, override_color=None,
           language_target=None):
    """gaussian_renderer/__init__.py:19-115.  language_target=(gt, mask) -- what
    Camera.get_language_feature returns (scene/cameras.py:58-92), e.g. from loss.LanguageFeatureCache
    -- additionally returns "language_l1" = l1_loss(language_feature_image * mask, gt * mask), the
    language loss of train.py:96-99, computed inside the rasterizer kernels."""
    screenspace_points = _screenspace_points(pc.get_xyz)

    tanfovx = math.tan(viewpoint_camera.FoVx * 0.5)
    tanfovy = math.tan(viewpoint_camera.FoVy * 0.5)
    raster_settings = GaussianRasterizationSettings(
        image_height=int(viewpoint_camera.image_height),
        image_width=int(viewpoint_camera.image_width),
        tanfovx=tanfovx,
        tanfovy=tanfovy,
        bg=bg_color,
        scale_modifier=scaling_modifier,
        viewmatrix=viewpoint_camera.world_view_transform,
        projmatrix=viewpoint_camera.full_proj_transform,
        sh_degree=pc.active_sh_degree,
        campos=viewpoint_camera.camera_center,
        prefiltered=False,
        debug=pipe.debug,
        include_feature=opt.include_feature,
    )
    rasterizer = GaussianRasterizer(raster_settings=raster_settings)

    if _fusable(pc, pipe, override_color, screenspace_points.device):
        lang_raw = pc.get_language_feature if opt.include_feature else None
        fused = rasterize_gaussians_fused(
            pc.get_xyz, screenspace_points, pc._features_dc, pc._features_rest, pc._opacity, pc._scaling,
            pc._rotation, lang_raw, raster_settings, with_visibility=True,
            language_target=language_target if opt.include_feature else None)
        rendered_image, language_feature_image, radii, visible = fused[:4]
        pkg = {"render": rendered_image,
               "language_feature_image": language_feature_image,
               "viewspace_points": screenspace_points,
               "visibility_filter": visible,  # radii > 0, from the preprocess kernel
               "radii": radii}
        if language_target is not None:
            pkg["language_l1"] = fused[4] if opt.include_feature else _l1(language_feature_image, *language_target)
        return pkg

    means3D = pc.get_xyz
    means2D = screenspace_points
    opacity = pc.get_opacity
    scales = rotations = cov3D_precomp = None
    if pipe.compute_cov3D_python:
        cov3D_precomp = pc.get_covariance(scaling_modifier)
    else:
        scales = pc.get_scaling
        rotations = pc.get_rotation
    shs = colors_precomp = None
    if override_color is None:
        if pipe.convert_SHs_python:
            shs_view = pc.get_features.transpose(1, 2).view(-1, 3, (pc.max_sh_degree + 1) ** 2)
            dir_pp = pc.get_xyz - viewpoint_camera.camera_center.repeat(pc.get_features.shape[0], 1)
            dir_pp_normalized = dir_pp / dir_pp.norm(dim=1, keepdim=True)
            sh2rgb = eval_sh(pc.active_sh_degree, shs_view, dir_pp_normalized)
            colors_precomp = torch.clamp_min(sh2rgb + 0.5, 0.0)
        else:
            shs = pc.get_features
    else:
        colors_precomp = override_color
    if opt.include_feature:
        ready = _native.language_ready.active()
        if ready is not None:
            # a pipelined / overlapped step (language_ready): the feature's update runs on another
            # stream; the fused path defers the feature inside the rasterizer, this path reads it
            # here, so the stream waits for the update first
            torch.cuda.current_stream().wait_event(ready)
        language_feature_precomp = pc.get_language_feature
        language_feature_precomp = language_feature_precomp / (
            language_feature_precomp.norm(dim=-1, keepdim=True) + 1e-9)
    else:
        language_feature_precomp = torch.zeros((1,), dtype=opacity.dtype, device=opacity.device)

    rendered_image, language_feature_image, radii = rasterizer(
        means3D=means3D, means2D=means2D, shs=shs, colors_precomp=colors_precomp,
        language_feature_precomp=language_feature_precomp, opacities=opacity, scales=scales,
        rotations=rotations, cov3D_precomp=cov3D_precomp)
    pkg = {"render": rendered_image,
           "language_feature_image": language_feature_image,
           "viewspace_points": screenspace_points,
           "visibility_filter": radii > 0,
           "radii": radii}
    if language_target is not None:
        pkg["language_l1"] = _l1(language_feature_image, *language_target)
    return pkg


def _l1(language_feature_image, gt, mask):
    """train.py:98 with utils/loss_utils.py:17-18, for the paths that do not fuse the loss."""
    return torch.abs(language_feature_image * mask - gt * mask).mean()
