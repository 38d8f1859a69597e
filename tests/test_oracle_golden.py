"""Pin the oracle against the reference's own outputs (tests/golden, made by make_golden.py from
/root/reference utils/sh_utils.py and utils/graphics_utils.py) and against analytic facts."""
import math
import os

import numpy as np
import pytest
import torch

from oracle import oracle
from langsplat_amd.camera import focal2fov, fov2focal, look_at_origin, make_camera

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def sh_gold():
    return np.load(os.path.join(GOLD, "sh_eval.npz"))


@pytest.mark.parametrize("deg", [0, 1, 2, 3])
def test_sh_eval_matches_reference(sh_gold, deg):
    """oracle SH basis == utils/sh_utils.py:eval_sh (fp32 vs the reference in fp64)."""
    sh = sh_gold[f"deg{deg}_sh"]            # (N, 3, 16)  reference layout [..., C, coeff]
    dirs_raw = sh_gold[f"deg{deg}_dirs_raw"]
    dirs = dirs_raw / np.linalg.norm(dirs_raw, axis=1, keepdims=True)
    ours = oracle.sh_eval(deg, np.transpose(sh, (0, 2, 1)), dirs)   # oracle takes (N, K, 3)
    ref = sh_gold[f"deg{deg}_value"]
    np.testing.assert_allclose(ours, ref, rtol=2e-5, atol=2e-6)


@pytest.mark.parametrize("deg", [0, 1, 2, 3])
def test_sh_backward_matches_reference_autograd(sh_gold, deg):
    """oracle SH backward (dsh, d direction through normalisation) == autograd of eval_sh(+0.5, clamp)."""
    sh = np.transpose(sh_gold[f"deg{deg}_sh"], (0, 2, 1))
    dirs_raw = sh_gold[f"deg{deg}_dirs_raw"]
    rgb = sh_gold[f"deg{deg}_rgb"]
    gout = sh_gold[f"deg{deg}_grad_out"]
    masked = np.where(rgb > 0, gout, 0.0)       # clamp_min(., 0) passes no gradient when clamped
    dsh, ddir = oracle.sh_backward(deg, sh, dirs_raw, masked)
    K = (deg + 1) ** 2
    ref_dsh = np.transpose(sh_gold[f"deg{deg}_grad_sh"], (0, 2, 1))
    np.testing.assert_allclose(dsh[:, :K], ref_dsh[:, :K], rtol=2e-5, atol=2e-6)
    assert np.all(dsh[:, K:] == 0)
    np.testing.assert_allclose(ddir, sh_gold[f"deg{deg}_grad_dirs_raw"], rtol=1e-4, atol=2e-5)


def test_rgb_sh_conversions(sh_gold):
    C0 = 0.28209479177387814
    np.testing.assert_allclose((sh_gold["rgb2sh_in"] - 0.5) / C0, sh_gold["rgb2sh_out"], rtol=1e-12)


def test_cameras_match_reference():
    """langsplat_amd.camera reproduces scene/cameras.py:48-57 + utils/graphics_utils.py bit for bit."""
    g = np.load(os.path.join(GOLD, "cameras.npz"))
    for n in range(int(g["count"])):
        W, H = int(g[f"c{n}_W"]), int(g[f"c{n}_H"])
        views, k = int(g[f"c{n}_views"]), int(g[f"c{n}_k"])
        fovy = math.radians(50.0)
        fovx = focal2fov(fov2focal(fovy, H), W)
        assert fovx == float(g[f"c{n}_fovx"])
        th = 2.0 * math.pi * k / views
        R, T = look_at_origin(np.array([4.0 * math.sin(th), 0.0, -4.0 * math.cos(th)]))
        np.testing.assert_array_equal(R, g[f"c{n}_R"])
        cam = make_camera(R, T, fovx, fovy, W, H)
        np.testing.assert_array_equal(cam.world_view_transform.numpy(), g[f"c{n}_world_view"])
        np.testing.assert_array_equal(cam.full_proj_transform.numpy(), g[f"c{n}_full_proj"])
        np.testing.assert_array_equal(cam.camera_center.numpy(), g[f"c{n}_center"])


def test_expf_restatement_accuracy():
    """The shared exp restatement is within 2 ulp of the true exp on the compositing domain."""
    xs = np.concatenate([np.linspace(-87.0, 0.0, 20001, dtype=np.float32),
                         -np.logspace(-8, 1.5, 2001).astype(np.float32)])
    ours = np.array([oracle.expf(float(x)) for x in xs], dtype=np.float32)
    ref = np.exp(xs.astype(np.float64))
    ulp = np.spacing(ref.astype(np.float32)).astype(np.float64)
    assert np.max(np.abs(ours - ref) / ulp) <= 2.0
    assert oracle.expf(0.0) == 1.0
    assert oracle.expf(-100.0) == 0.0


def test_expf_render_restatement_accuracy():
    """The compositing loops' exp (one-constant range reduction) is within 2 ulp of the true exp
    wherever they use it (power >= ln(1/255) - 0.01 > -6), and beyond, down to -20."""
    xs = np.concatenate([np.linspace(-20.0, 0.0, 40001, dtype=np.float32),
                         -np.logspace(-8, 1.3, 2001).astype(np.float32)])
    ours = np.array([oracle.expf_render(float(x)) for x in xs], dtype=np.float32)
    ref = np.exp(xs.astype(np.float64))
    ulp = np.spacing(ref.astype(np.float32)).astype(np.float64)
    assert np.max(np.abs(ours - ref) / ulp) <= 2.0
    assert oracle.expf_render(0.0) == 1.0


def test_cov3d_is_rssr():
    """Sigma = R S S^T R^T (scene/gaussian_model.py:27-31 with utils/general_utils.py:78-110)."""
    g = torch.Generator().manual_seed(3)
    s = torch.rand((32, 3), generator=g, dtype=torch.float64) * 0.5 + 0.01
    q = torch.nn.functional.normalize(torch.randn((32, 4), generator=g, dtype=torch.float64))
    r, x, y, z = q.unbind(-1)
    R = torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y),
                     2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x),
                     2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], -1).reshape(-1, 3, 3)
    L = R @ torch.diag_embed(s * 1.7)
    S = L @ L.transpose(1, 2)
    ref = torch.stack([S[:, 0, 0], S[:, 0, 1], S[:, 0, 2], S[:, 1, 1], S[:, 1, 2], S[:, 2, 2]], -1).numpy()
    ours = oracle.cov3d(s.numpy(), 1.7, q.numpy())
    np.testing.assert_allclose(ours, ref, rtol=2e-5, atol=1e-7)


def test_cov3d_backward_matches_autograd():
    g = torch.Generator().manual_seed(4)
    s = (torch.rand((16, 3), generator=g, dtype=torch.float64) * 0.5 + 0.05).requires_grad_(True)
    q = torch.nn.functional.normalize(torch.randn((16, 4), generator=g, dtype=torch.float64)).requires_grad_(True)
    dcov = torch.randn((16, 6), generator=g, dtype=torch.float64)
    r, x, y, z = q.unbind(-1)
    R = torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y),
                     2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x),
                     2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], -1).reshape(-1, 3, 3)
    L = R @ torch.diag_embed(s)
    S = L @ L.transpose(1, 2)
    packed = torch.stack([S[:, 0, 0], S[:, 0, 1], S[:, 0, 2], S[:, 1, 1], S[:, 1, 2], S[:, 2, 2]], -1)
    (packed * dcov).sum().backward()
    ds, dr = oracle.cov3d_backward(s.detach().numpy(), 1.0, q.detach().numpy(), dcov.numpy())
    np.testing.assert_allclose(ds, s.grad.numpy(), rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(dr, q.grad.numpy(), rtol=1e-4, atol=1e-6)
