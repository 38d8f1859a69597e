"""render() with pipe.convert_SHs_python and pipe.compute_cov3D_python.

gaussian_renderer/__init__.py:61-80: with compute_cov3D_python the covariance comes from
pc.get_covariance (scene/gaussian_model.py:27-31,163-164: L = R(normalised q) diag(s * mod),
strip_symmetric(L L^T)) and reaches the rasterizer as cov3D_precomp; with convert_SHs_python the
colours come from eval_sh(+0.5, clamp_min 0) on the view directions and reach it as
colors_precomp.  Both switches run through render() here, on GPU torch ops plus the HIP rasterizer.

Checked against the oracle: its forward on the same colors_precomp / cov3D_precomp / opacity /
language tensors (computed by the same torch ops) must give the same images bit for bit, and its
gradients w.r.t. those inputs, chained to GaussianModel's raw parameters by torch autograd through
the same ops, must match the raw-parameter gradients render() + backward produce.
"""
import numpy as np
import pytest
import torch

from langsplat_amd.render import eval_sh, render
from langsplat_amd.synthetic import make_cameras, make_gaussians
from oracle import oracle
from tests.scenes import grad_seed, settings_for
from tests.test_gpu_fused import _Model, _Opt
from tests.test_gpu_parity import assert_grad_close

pytestmark = pytest.mark.gpu
DEV = "cuda"
NAMES = ("xyz", "features_dc", "features_rest", "scaling", "rotation", "opacity", "language_feature")


def build_covariance(scaling, scaling_modifier, rotation):
    """scene/gaussian_model.py:27-31 build_covariance_from_scaling_rotation with
    utils/general_utils.py:78-110 (build_rotation normalises q; strip_symmetric keeps the upper 6)."""
    q = rotation / torch.sqrt(rotation[:, 0] ** 2 + rotation[:, 1] ** 2 + rotation[:, 2] ** 2 +
                              rotation[:, 3] ** 2)[:, None]
    r, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R = torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y),
                     2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x),
                     2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], -1).reshape(-1, 3, 3)
    L = R @ torch.diag_embed(scaling_modifier * scaling)
    S = L @ L.transpose(1, 2)
    return torch.stack([S[:, 0, 0], S[:, 0, 1], S[:, 0, 2], S[:, 1, 1], S[:, 1, 2], S[:, 2, 2]], -1)


class _CovModel(_Model):
    def get_covariance(self, scaling_modifier=1.0):
        return build_covariance(self.get_scaling, scaling_modifier, self._rotation)


class _PyPipe:
    convert_SHs_python = True
    compute_cov3D_python = True
    debug = False


def _python_inputs(m, cam, scaling_modifier):
    """What render() computes under both switches (gaussian_renderer/__init__.py:55-91)."""
    cov = m.get_covariance(scaling_modifier)
    feats = m.get_features
    shs_view = feats.transpose(1, 2).view(-1, 3, (m.max_sh_degree + 1) ** 2)
    dir_pp = m.get_xyz - cam.camera_center.repeat(feats.shape[0], 1)
    dirs = dir_pp / dir_pp.norm(dim=1, keepdim=True)
    colors = torch.clamp_min(eval_sh(m.active_sh_degree, shs_view, dirs) + 0.5, 0.0)
    lf = m.get_language_feature
    lang = lf / (lf.norm(dim=-1, keepdim=True) + 1e-9)
    return dict(means3D=m.get_xyz, opacities=m.get_opacity, colors_precomp=colors, cov3D_precomp=cov,
                language_feature_precomp=lang)


@pytest.mark.parametrize("deg,mod", [(3, 1.0), (1, 1.25)])
def test_render_python_sh_and_cov3d_switches_match_oracle(deg, mod):
    W, H = 96, 64
    g = make_gaussians(1500, seed=14, sh_degree=3, scale_range=(0.03, 0.2))
    cam = make_cameras(1, W, H, device=DEV)[0]
    m = _CovModel(g, DEV)
    m.active_sh_degree = deg
    gc, gl = (t.to(DEV) for t in grad_seed(H, W, seed=15))
    pkg = render(cam, m, _PyPipe, torch.zeros(3, device=DEV), _Opt, scaling_modifier=mod)
    ((pkg["render"] * gc).sum() + (pkg["language_feature_image"] * gl).sum()).backward()
    got = {n: getattr(m, "_" + n).grad.detach().cpu().numpy() for n in NAMES}

    # oracle on the same precomputed inputs; cov3D_precomp already carries the scaling modifier
    m2 = _CovModel(g, DEV)
    m2.active_sh_degree = deg
    inp = _python_inputs(m2, cam, mod)
    st = settings_for(cam.to("cpu"), sh_degree=deg, scale_modifier=mod)
    run = oracle.forward(st, **{k: v.detach().cpu() for k, v in inp.items()})
    np.testing.assert_array_equal(pkg["render"].detach().cpu().numpy(), run.color)
    np.testing.assert_array_equal(pkg["language_feature_image"].detach().cpu().numpy(), run.language)
    np.testing.assert_array_equal(pkg["radii"].cpu().numpy(), run.radii)
    ref = run.backward(gc.cpu(), gl.cpu())
    keys = ("means3D", "opacities", "colors_precomp", "cov3D_precomp", "language_feature_precomp")
    torch.autograd.backward([inp[k] for k in keys],
                            [torch.from_numpy(ref[k]).to(DEV).view_as(inp[k]) for k in keys])
    for n in NAMES:
        want = getattr(m2, "_" + n).grad.detach().cpu().numpy()
        assert_grad_close(n, got[n], want)
    assert np.abs(got["features_rest"]).sum() > 0 if deg > 0 else True
