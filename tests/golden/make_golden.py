"""Generate golden vectors from the reference's own (importable, CPU) Python code.

Run in the build container only (the reference is not on the GPU box):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Imports from /root/reference (SURVEY.md §8c "what is importable"):
  - utils/sh_utils.py: eval_sh (deg 0-3), RGB2SH / SH2RGB, constants
  - utils/graphics_utils.py: getWorld2View2, getProjectionMatrix, fov2focal, focal2fov
Camera matrices are assembled exactly as scene/cameras.py:54-57 does (that module itself does not
import here: scene/__init__.py pulls plyfile/simple_knn).  Outputs are plain .npz data files.
"""
import math
import os
import sys

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REF)
sys.dont_write_bytecode = True

from utils.graphics_utils import focal2fov, fov2focal, getProjectionMatrix, getWorld2View2  # noqa: E402
from utils.sh_utils import RGB2SH, SH2RGB, eval_sh  # noqa: E402


def sh_fixtures():
    g = torch.Generator().manual_seed(1234)
    N = 64
    out = {}
    for deg in range(4):
        K = (deg + 1) ** 2
        sh = torch.randn((N, 3, 16), generator=g, dtype=torch.float64) * 0.5   # [..., C, coeff]
        dirs_raw = torch.randn((N, 3), generator=g, dtype=torch.float64)
        gout = torch.randn((N, 3), generator=g, dtype=torch.float64)
        sh.requires_grad_(True)
        dirs_raw.requires_grad_(True)
        dirs = dirs_raw / dirs_raw.norm(dim=1, keepdim=True)
        val = eval_sh(deg, sh, dirs)
        # gaussian_renderer/__init__.py:80 convention
        rgb = torch.clamp_min(val + 0.5, 0.0)
        (rgb * gout).sum().backward()
        out[f"deg{deg}_sh"] = sh.detach().numpy()
        out[f"deg{deg}_dirs_raw"] = dirs_raw.detach().numpy()
        out[f"deg{deg}_value"] = val.detach().numpy()
        out[f"deg{deg}_rgb"] = rgb.detach().numpy()
        out[f"deg{deg}_grad_out"] = gout.numpy()
        out[f"deg{deg}_grad_sh"] = sh.grad.numpy()
        out[f"deg{deg}_grad_dirs_raw"] = (dirs_raw.grad if dirs_raw.grad is not None else torch.zeros_like(dirs_raw)).numpy()
        out[f"deg{deg}_K"] = np.int64(K)
    rgb = torch.rand((16, 3), generator=g, dtype=torch.float64)
    out["rgb2sh_in"] = rgb.numpy()
    out["rgb2sh_out"] = RGB2SH(rgb).numpy()
    out["sh2rgb_out"] = SH2RGB(RGB2SH(rgb)).numpy()
    np.savez(os.path.join(OUT, "sh_eval.npz"), **out)


def look_at_origin(position):
    c = np.asarray(position, dtype=np.float64)
    z = -c / np.linalg.norm(c)
    x = np.cross(np.array([0.0, 1.0, 0.0]), z)
    x /= np.linalg.norm(x)
    y = np.cross(z, x)
    R = np.stack([x, y, z], axis=1)
    return R, -R.T @ c


def camera_fixtures():
    out = {}
    cases = [(400, 300, 1), (1280, 720, 1), (1920, 1080, 8), (64, 48, 3), (37, 29, 2)]
    n = 0
    for (W, H, views) in cases:
        fovy = math.radians(50.0)
        fovx = focal2fov(fov2focal(fovy, H), W)
        for k in range(views):
            th = 2.0 * math.pi * k / views
            pos = np.array([4.0 * math.sin(th), 0.0, -4.0 * math.cos(th)])
            R, T = look_at_origin(pos)
            # scene/cameras.py:48-57 with trans = 0, scale = 1
            wv = torch.tensor(getWorld2View2(R, T, np.array([0.0, 0.0, 0.0]), 1.0)).transpose(0, 1)
            proj = getProjectionMatrix(znear=0.01, zfar=100.0, fovX=fovx, fovY=fovy).transpose(0, 1)
            full = wv.unsqueeze(0).bmm(proj.unsqueeze(0)).squeeze(0)
            center = wv.inverse()[3, :3]
            out[f"c{n}_W"] = np.int64(W)
            out[f"c{n}_H"] = np.int64(H)
            out[f"c{n}_views"] = np.int64(views)
            out[f"c{n}_k"] = np.int64(k)
            out[f"c{n}_R"] = R
            out[f"c{n}_T"] = T
            out[f"c{n}_fovx"] = np.float64(fovx)
            out[f"c{n}_fovy"] = np.float64(fovy)
            out[f"c{n}_world_view"] = wv.numpy()
            out[f"c{n}_full_proj"] = full.numpy()
            out[f"c{n}_center"] = center.numpy()
            n += 1
    out["count"] = np.int64(n)
    np.savez(os.path.join(OUT, "cameras.npz"), **out)


if __name__ == "__main__":
    sh_fixtures()
    camera_fixtures()
    print("wrote", sorted(f for f in os.listdir(OUT) if f.endswith(".npz")))
