"""The exact step bench.py times, against the oracle, at full size.

bench.py times LangSplat's language-feature train step (train.py:76-104): render() on GaussianModel's
raw parameters (activations inside k_preprocess), the masked L1 of train.py:96-99 inside the
compositing kernel (render(..., language_target=(gt, mask))["language_l1"]), and loss.backward()
with every geometry parameter frozen (scene/gaussian_model.py:203-217).  That backward is the
5-value k_render_backward<false, true, false, false>: its per-pixel seed comes from the forward's
sign/mask code bytes, it reads the forward's cover masks, and it accumulates into the gradient
records the forward cleared (LSR_FWD_ZERO_GRAD_RECORDS / LSR_BWD_RECORDS_ZEROED).

The oracle side: oracle.activate of the raw parameters (bit-identical to the kernels' activations),
oracle.forward (whose images the GPU reproduces bit for bit, asserted here), the seed
dL/dlang = sign(f m - gt m) m / (3 H W) that autograd forms for train.py:98's expression, computed
in float32 from the oracle's own image, oracle backward, and the language normalisation's backward
(oracle.activate_backward).  Gradient tolerance as tests/test_gpu_parity.py (1e-4 relative with a
1e-2 * max floor); the loss within 2e-6 of the float64 sum over the oracle image.

Configs: C2 and C3 (BASELINE.json configs[1], [2], camera 0) and one off-axis camera of C4
(make_cameras(8, ...)[3]: 135 degrees round the circle) -- the per-GPU view of the multi-GPU bench.
"""
import numpy as np
import pytest
import torch

from langsplat_amd.synthetic import CONFIGS, make_cameras, make_gaussians
from oracle import oracle
from tests.scenes import settings_for
from tests.test_gpu_fused import _Model, _Opt, _Pipe
from tests.test_gpu_parity import assert_grad_close

pytestmark = pytest.mark.gpu
DEV = "cuda"


def bench_target(H, W, view):
    """bench.py's synthetic language target for `view`: a unit-vector map and a 90 % mask."""
    gen = torch.Generator().manual_seed(100 + view)
    gt = torch.nn.functional.normalize(torch.randn((3, H, W), generator=gen), dim=0)
    mask = torch.rand((1, H, W), generator=gen) < 0.9
    return gt, mask


def oracle_language_step(g, cam, gt, mask):
    """Oracle forward + the language step's backward; returns (run, loss, d_lang_raw, d_means2D)."""
    c = cam
    st = settings_for(c, sh_degree=3)
    a_op, a_sc, a_rot, a_lang = oracle.activate(oracle.RAW_ALL, g.opacity, g.scaling, g.rotation,
                                                g.language_feature)
    shs = torch.cat((g.features_dc, g.features_rest), dim=1).contiguous()
    run = oracle.forward(st, means3D=g.xyz, opacities=a_op, scales=a_sc, rotations=a_rot, shs=shs,
                         language_feature_precomp=a_lang)
    H, W = run.H, run.W
    m = mask.numpy().astype(np.float32).reshape(1, H, W)
    gtn = gt.numpy().astype(np.float32)
    d = run.language * m - gtn * m  # float32, as torch evaluates lang * mask - gt * mask
    loss = float(np.abs(d.astype(np.float64)).sum() / (3 * H * W))
    # autograd of mean(abs(d)): (1 / numel) * sign(d), then the mask multiply
    seed = (np.float32(1.0) / np.float32(3 * H * W)) * np.sign(d).astype(np.float32) * m
    ref = run.backward(np.zeros_like(seed), seed.astype(np.float32))
    _, _, _, d_lang = oracle.activate_backward(oracle.RAW_LANGUAGE, (None, None, None, g.language_feature),
                                               (None, None, None, ref["language_feature_precomp"]))
    return run, loss, d_lang, ref["means2D"]


def gpu_language_step(g, cam, gt, mask, monkeypatch):
    """bench.py's step() on the fused path: render with the fused loss, loss.backward()."""
    from langsplat_amd.render import render
    monkeypatch.setenv("LANGSPLAT_AMD_FUSED", "1")
    m = _Model(g, DEV)
    for n in ("xyz", "features_dc", "features_rest", "scaling", "rotation", "opacity"):
        getattr(m, "_" + n).requires_grad_(False)
    pkg = render(cam.to(DEV), m, _Pipe, torch.zeros(3, device=DEV), _Opt,
                 language_target=(gt.to(DEV), mask.to(DEV)))
    loss = pkg["language_l1"]
    loss.backward()
    torch.cuda.synchronize()
    return (pkg["render"].detach().cpu().numpy(), pkg["language_feature_image"].detach().cpu().numpy(),
            pkg["radii"].cpu().numpy(), float(loss.item()), m._language_feature.grad.cpu().numpy(),
            pkg["viewspace_points"].grad.cpu().numpy())


@pytest.mark.parametrize("cfg,view", [("C2", 0), ("C3", 0), ("C4", 3)])
def test_timed_language_step_matches_oracle(cfg, view, monkeypatch):
    c = CONFIGS[cfg]
    P, W, H = c["P"], c["width"], c["height"]
    g = make_gaussians(P, seed=0)
    cam = make_cameras(c["views"], W, H)[view]
    gt, mask = bench_target(H, W, view)
    run, loss_ref, d_lang_ref, d_m2_ref = oracle_language_step(g, cam, gt, mask)
    color, lang, radii, loss, d_lang, d_m2 = gpu_language_step(g, cam, gt, mask, monkeypatch)
    assert run.blends > 0
    np.testing.assert_array_equal(radii, run.radii)
    np.testing.assert_array_equal(color, run.color)
    np.testing.assert_array_equal(lang, run.language)
    assert abs(loss - loss_ref) <= 2e-6 * loss_ref, (loss, loss_ref)
    assert_grad_close("language_feature (raw)", d_lang, d_lang_ref)
    assert_grad_close("viewspace_points", d_m2, d_m2_ref)
    assert np.abs(d_lang).sum() > 0
