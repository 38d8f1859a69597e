"""Dense PyTorch-autograd restatement of the rasterizer -- an INDEPENDENT check of the C oracle.

TEST INFRASTRUCTURE ONLY (see oracle/lsr_oracle.c header).  Where lsr_oracle.c restates the
upstream kernels line by line (per-pixel loops, hand-derived backward with T recovered by
division), this file writes the same model as dense tensor algebra per tile -- alpha matrix,
cumulative-product transmittance, termination mask -- and lets torch.autograd derive every
gradient.  Agreement of the two (tests/test_torch_reference.py) pins the oracle's hand-written
backward and the compositing semantics; both follow SURVEY.md Appendix A and the reference call
site gaussian_renderer/__init__.py:19-115.

Semantics encoded explicitly (the upstream choices the autograd graph would not make by itself):
  - alpha = min(0.99, o*G) is straight-through: d alpha / d(o G) = 1 even when clamped;
  - the EWA window clamp |t.x/t.z| <= 1.3 tan(fov/2) passes no gradient to t when active;
  - discrete decisions (culling, radius, tile rectangles, depth order, alpha/T cut-offs) carry
    no gradient; means2D receives dL/d(NDC position) through an additive zero sink.
Small inputs only (python loop over tiles).
"""
from __future__ import annotations

import math

import torch

SH_C0 = 0.28209479177387814
SH_C1 = 0.4886025119029199
SH_C2 = [1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396]
SH_C3 = [-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
         1.445305721320277, -0.5900435899266435]


def sh_to_rgb(deg, sh, dirs):
    """sh: (P, K, 3), dirs: (P, 3) unit -> (P, 3); utils/sh_utils.py:57-112 basis."""
    x, y, z = dirs[:, 0:1], dirs[:, 1:2], dirs[:, 2:3]
    res = SH_C0 * sh[:, 0]
    if deg > 0:
        res = res - SH_C1 * y * sh[:, 1] + SH_C1 * z * sh[:, 2] - SH_C1 * x * sh[:, 3]
    if deg > 1:
        xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
        res = (res + SH_C2[0] * xy * sh[:, 4] + SH_C2[1] * yz * sh[:, 5] + SH_C2[2] * (2 * zz - xx - yy) * sh[:, 6]
               + SH_C2[3] * xz * sh[:, 7] + SH_C2[4] * (xx - yy) * sh[:, 8])
    if deg > 2:
        res = (res + SH_C3[0] * y * (3 * xx - yy) * sh[:, 9] + SH_C3[1] * xy * z * sh[:, 10]
               + SH_C3[2] * y * (4 * zz - xx - yy) * sh[:, 11] + SH_C3[3] * z * (2 * zz - 3 * xx - 3 * yy) * sh[:, 12]
               + SH_C3[4] * x * (4 * zz - xx - yy) * sh[:, 13] + SH_C3[5] * z * (xx - yy) * sh[:, 14]
               + SH_C3[6] * x * (xx - 3 * yy) * sh[:, 15])
    return res


def rot_matrix(q):
    r, x, y, z = q.unbind(-1)
    return torch.stack([
        1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y),
        2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x),
        2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], -1).reshape(-1, 3, 3)


def rasterize(settings, means3D, means2D, opacities, shs=None, colors_precomp=None, language_feature=None,
              scales=None, rotations=None, cov3D_precomp=None):
    """Returns (color (3,H,W), language (3,H,W), radii (P,), n_contrib (H,W))."""
    H, W = int(settings.image_height), int(settings.image_width)
    dt = means3D.dtype
    view = settings.viewmatrix.to(dt)
    proj = settings.projmatrix.to(dt)
    campos = settings.campos.to(dt)
    bg = settings.bg.to(dt)
    P = means3D.shape[0]
    ones = torch.ones((P, 1), dtype=dt)
    ph = torch.cat([means3D, ones], 1)
    p_view = ph @ view
    p_hom = ph @ proj
    p_w = 1.0 / (p_hom[:, 3:4] + 1e-7)
    p_proj = p_hom[:, :2] * p_w + means2D[:, :2]
    if cov3D_precomp is not None:
        c6 = cov3D_precomp
        Sigma = torch.stack([c6[:, 0], c6[:, 1], c6[:, 2], c6[:, 1], c6[:, 3], c6[:, 4],
                             c6[:, 2], c6[:, 4], c6[:, 5]], -1).reshape(-1, 3, 3)
    else:
        Mm = rot_matrix(rotations) * (scales * settings.scale_modifier)[:, None, :]
        Sigma = Mm @ Mm.transpose(1, 2)
    t = p_view[:, :3]
    tanx, tany = float(settings.tanfovx), float(settings.tanfovy)
    fx, fy = W / (2 * tanx), H / (2 * tany)
    limx, limy = 1.3 * tanx, 1.3 * tany
    txtz, tytz = t[:, 0] / t[:, 2], t[:, 1] / t[:, 2]
    cx_ = (txtz < -limx) | (txtz > limx)
    cy_ = (tytz < -limy) | (tytz > limy)
    tx = torch.where(cx_, (txtz.clamp(-limx, limx) * t[:, 2]).detach(), t[:, 0])
    ty = torch.where(cy_, (tytz.clamp(-limy, limy) * t[:, 2]).detach(), t[:, 1])
    tz = t[:, 2]
    zero = torch.zeros_like(tz)
    J = torch.stack([fx / tz, zero, -fx * tx / (tz * tz), zero, fy / tz, -fy * ty / (tz * tz)], -1).reshape(-1, 2, 3)
    Wr = view[:3, :3].T  # world->camera rotation
    A = J @ Wr
    cov2 = A @ Sigma @ A.transpose(1, 2)
    a = cov2[:, 0, 0] + 0.3
    b = cov2[:, 0, 1]
    c = cov2[:, 1, 1] + 0.3
    det = a * c - b * b
    conic = torch.stack([c / det, -b / det, a / det], -1)
    # discrete decisions (no gradient), fp32 like the kernels
    with torch.no_grad():
        det32 = det.float()
        mid = 0.5 * (a + c).float()
        lam = mid + torch.sqrt(torch.clamp(mid * mid - det32, min=0.1))
        radius = torch.ceil(3.0 * torch.sqrt(lam))
        visible = (p_view[:, 2].float() > 0.2) & (det32 != 0)
    pix = torch.stack([((p_proj[:, 0] + 1.0) * W - 1.0) * 0.5, ((p_proj[:, 1] + 1.0) * H - 1.0) * 0.5], -1)
    if shs is not None:
        d = means3D - campos[None]
        dirs = d / d.norm(dim=1, keepdim=True)
        raw = sh_to_rgb(int(settings.sh_degree), shs, dirs) + 0.5
        rgb = torch.clamp_min(raw, 0.0)
    else:
        rgb = colors_precomp
    feat = bool(settings.include_feature) and language_feature is not None and language_feature.numel() == 3 * P
    lang = language_feature if feat else torch.zeros((P, 3), dtype=dt)
    opac = opacities.reshape(-1)

    gx, gy = (W + 15) // 16, (H + 15) // 16
    with torch.no_grad():
        r_i = radius.to(torch.int64)
        pxf = pix.detach().float()
        rminx = torch.clamp(torch.trunc((pxf[:, 0] - r_i) / 16).to(torch.int64), 0, gx)
        rminy = torch.clamp(torch.trunc((pxf[:, 1] - r_i) / 16).to(torch.int64), 0, gy)
        rmaxx = torch.clamp(torch.trunc((pxf[:, 0] + r_i + 15) / 16).to(torch.int64), 0, gx)
        rmaxy = torch.clamp(torch.trunc((pxf[:, 1] + r_i + 15) / 16).to(torch.int64), 0, gy)
        visible &= (rmaxx - rminx) * (rmaxy - rminy) > 0
        radii = torch.where(visible, r_i, torch.zeros_like(r_i)).to(torch.int32)
        depth = p_view[:, 2].detach().float()

    n_contrib = torch.zeros((H, W), dtype=torch.int64)
    tiles_c, tiles_f = {}, {}
    for ty_ in range(gy):
        for tx_ in range(gx):
            with torch.no_grad():
                sel = visible & (rminx <= tx_) & (tx_ < rmaxx) & (rminy <= ty_) & (ty_ < rmaxy)
                ids = torch.nonzero(sel).flatten()
                if ids.numel():
                    order = sorted(ids.tolist(), key=lambda i: (depth[i].item(), i))
                    ids = torch.tensor(order, dtype=torch.int64)
            x0, y0 = tx_ * 16, ty_ * 16
            xs = torch.arange(x0, min(x0 + 16, W), dtype=dt)
            ys = torch.arange(y0, min(y0 + 16, H), dtype=dt)
            PY, PX = torch.meshgrid(ys, xs, indexing="ij")
            npx = PX.numel()
            if ids.numel() == 0:
                tiles_c[(ty_, tx_)] = (bg[:, None] * torch.ones((1, npx), dtype=dt)).reshape(3, *PX.shape)
                tiles_f[(ty_, tx_)] = torch.zeros((3, *PX.shape), dtype=dt)
                continue
            dx = pix[ids, 0][:, None] - PX.reshape(1, -1)
            dy = pix[ids, 1][:, None] - PY.reshape(1, -1)
            co = conic[ids]
            power = -0.5 * (co[:, 0:1] * dx * dx + co[:, 2:3] * dy * dy) - co[:, 1:2] * dx * dy
            G = torch.exp(power)
            oG = opac[ids][:, None] * G
            alpha = oG - (oG - torch.clamp(oG, max=0.99)).detach()
            with torch.no_grad():
                valid = (power <= 0) & (alpha >= 1.0 / 255.0)
                om = torch.where(valid, 1.0 - alpha, torch.ones_like(alpha))
                Tb = torch.cumprod(torch.cat([torch.ones_like(om[:1]), om[:-1]], 0), 0)
                term = valid & (Tb * (1.0 - alpha) < 1e-4)
                K = alpha.shape[0]
                idx = torch.arange(K)[:, None].expand_as(alpha)
                first = torch.where(term, idx, torch.full_like(idx, K)).min(0).values
                blended = valid & (idx < first[None])
                last = torch.where(blended, idx + 1, torch.zeros_like(idx)).max(0).values
            om_b = torch.where(blended, 1.0 - alpha, torch.ones_like(alpha))
            T_before = torch.cumprod(torch.cat([torch.ones_like(om_b[:1]), om_b[:-1]], 0), 0)
            w = torch.where(blended, alpha * T_before, torch.zeros_like(alpha))
            Tf = torch.prod(om_b, 0)
            cimg = (w[:, None, :] * rgb[ids][:, :, None]).sum(0) + Tf[None] * bg[:, None]
            fimg = (w[:, None, :] * lang[ids][:, :, None]).sum(0)
            tiles_c[(ty_, tx_)] = cimg.reshape(3, *PX.shape)
            tiles_f[(ty_, tx_)] = fimg.reshape(3, *PX.shape)
            n_contrib[y0:y0 + PX.shape[0], x0:x0 + PX.shape[1]] = last.reshape(PX.shape)
    color = torch.cat([torch.cat([tiles_c[(j, i)] for i in range(gx)], 2) for j in range(gy)], 1)
    language = torch.cat([torch.cat([tiles_f[(j, i)] for i in range(gx)], 2) for j in range(gy)], 1)
    return color, language, radii, n_contrib
