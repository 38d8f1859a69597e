"""Oracle rendering: analytic known-answer cases and agreement with the
independent dense-autograd restatement (oracle/torch_ref.py), forward and backward."""
import math

import numpy as np
import pytest
import torch

from oracle import oracle, torch_ref
from tests.scenes import grad_seed, scene, settings_for
from langsplat_amd.camera import look_at_origin, make_camera


def _cam(W=64, H=48):
    fovy = math.radians(50.0)
    fovx = 2 * math.atan(math.tan(fovy / 2) * W / H)
    R, T = look_at_origin(np.array([0.0, 0.0, -4.0]))
    return make_camera(R, T, fovx, fovy, W, H)


def _single(mean, scale, opacity, color, W=64, H=48, bg=(0.0, 0.0, 0.0)):
    st = settings_for(_cam(W, H), sh_degree=0, bg=bg)
    inp = dict(means3D=torch.tensor([mean], dtype=torch.float32),
               opacities=torch.tensor([[opacity]], dtype=torch.float32),
               colors_precomp=torch.tensor([color], dtype=torch.float32),
               language_feature_precomp=torch.tensor([[0.6, 0.0, 0.8]], dtype=torch.float32),
               scales=torch.tensor([[scale] * 3], dtype=torch.float32),
               rotations=torch.tensor([[1.0, 0.0, 0.0, 0.0]], dtype=torch.float32))
    return st, inp


def test_single_isotropic_gaussian_centre_pixel():
    """A Gaussian projected exactly on pixel (31.5,23.5)'s neighbourhood: alpha = min(.99, o*G)."""
    st, inp = _single([0.0, 0.0, 0.0], 0.05, 0.5, [1.0, 0.5, 0.25])
    run = oracle.forward(st, **inp)
    xy = run.get("xy")[0]
    co = run.get("conic_opacity")[0]
    # centre of a 64x48 image at NDC 0 is pixel (31.5, 23.5)
    assert abs(xy[0] - 31.5) < 1e-5 and abs(xy[1] - 23.5) < 1e-5
    px, py = 31, 23
    dx, dy = xy[0] - px, xy[1] - py
    G = math.exp(-0.5 * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy)
    alpha = min(0.99, 0.5 * G)
    np.testing.assert_allclose(run.color[:, py, px], alpha * np.array([1.0, 0.5, 0.25]), rtol=1e-5)
    np.testing.assert_allclose(run.language[:, py, px], alpha * np.array([0.6, 0.0, 0.8]), rtol=1e-5)
    assert run.get("n_contrib")[py, px] == 1
    np.testing.assert_allclose(run.get("final_T")[py, px], 1 - alpha, rtol=1e-6)
    assert run.radii[0] > 0


def test_opacity_clamp_and_background():
    st, inp = _single([0.0, 0.0, 0.0], 1.5, 1.0, [1.0, 1.0, 1.0], bg=(0.2, 0.4, 0.6))
    run = oracle.forward(st, **inp)
    # near the centre G ~ 1 so alpha clamps at 0.99: colour = 0.99 + 0.01 * bg
    np.testing.assert_allclose(run.color[:, 23, 31], 0.99 + 0.01 * np.array([0.2, 0.4, 0.6]), rtol=1e-4)
    # language has no background term
    st2, inp2 = _single([0.0, 0.0, 0.0], 0.02, 1.0, [1.0, 1.0, 1.0], bg=(0.2, 0.4, 0.6))
    run2 = oracle.forward(st2, **inp2)
    np.testing.assert_array_equal(run2.color[:, 0, 0], np.array([0.2, 0.4, 0.6], np.float32))
    assert np.all(run2.language[:, 0, 0] == 0)


def test_near_plane_cull():
    """z_view <= 0.2 -> radius 0, no tiles (camera at z=-4: a point at z=-3.85 is 0.15 deep)."""
    st, inp = _single([0.0, 0.0, -3.85], 0.05, 0.5, [1.0, 1.0, 1.0])
    run = oracle.forward(st, **inp)
    assert run.radii[0] == 0 and run.num_rendered == 0
    assert np.all(run.color == 0)


def test_low_alpha_skip():
    """alpha < 1/255 contributes nothing and is not counted as a contributor."""
    st, inp = _single([0.0, 0.0, 0.0], 0.05, 1.0 / 300.0, [1.0, 1.0, 1.0])
    run = oracle.forward(st, **inp)
    assert run.radii[0] > 0 and run.num_rendered > 0
    assert np.all(run.color == 0) and np.all(run.get("n_contrib") == 0)


def test_termination_at_T_1e4():
    """Front-to-back stops once T*(1-alpha) < 1e-4; later Gaussians are not blended."""
    W, H = 32, 32
    st = settings_for(_cam(W, H), sh_degree=0)
    n = 4
    means = torch.tensor([[0.0, 0.0, -1.0 + 0.1 * k] for k in range(n)], dtype=torch.float32)
    inp = dict(means3D=means, opacities=torch.full((n, 1), 0.99), colors_precomp=torch.eye(3)[[0, 1, 2, 0]],
               language_feature_precomp=torch.zeros((n, 3)), scales=torch.full((n, 3), 0.5),
               rotations=torch.tensor([[1.0, 0.0, 0.0, 0.0]] * n))
    run = oracle.forward(st, **inp)
    # alpha = 0.99 at the centre: T = 1 -> 0.01 -> 1e-4 (=T*(1-a) 1e-4 is not < 1e-4 in fp32? check)
    nc = run.get("n_contrib")[16, 16]
    T = run.get("final_T")[16, 16]
    assert nc in (1, 2)
    assert T >= 1e-4
    c = run.color[:, 16, 16]
    assert c[2] == 0.0  # third Gaussian (blue) never blended


def test_tile_lists_sorted_by_depth_then_id():
    st, inp = scene(P=400, W=64, H=48, seed=5)
    run = oracle.forward(st, **inp)
    pl = run.get("point_list")
    rg = run.get("ranges")
    depth = run.get("depth")
    for t in range(rg.shape[0]):
        seg = pl[rg[t, 0]:rg[t, 1]]
        keys = list(zip(depth[seg].tolist(), seg.tolist()))
        assert keys == sorted(keys)
    assert rg[-1, 1] <= run.num_rendered
    assert int(run.get("tiles_touched").sum()) == run.num_rendered


def test_equal_depth_ties_break_by_id():
    """Two Gaussians at identical depth: the lower id is composited first (stable sort)."""
    st = settings_for(_cam(32, 32), sh_degree=0)
    means = torch.tensor([[0.0, 0.0, 0.0], [0.01, 0.0, 0.0]], dtype=torch.float32)
    inp = dict(means3D=means, opacities=torch.full((2, 1), 0.5), colors_precomp=torch.eye(3)[:2],
               language_feature_precomp=torch.zeros((2, 3)), scales=torch.full((2, 3), 0.2),
               rotations=torch.tensor([[1.0, 0.0, 0.0, 0.0]] * 2))
    run = oracle.forward(st, **inp)
    d = run.get("depth")
    assert d[0] == d[1]
    pl = run.get("point_list")
    rg = run.get("ranges")
    for t in range(rg.shape[0]):
        seg = pl[rg[t, 0]:rg[t, 1]].tolist()
        if len(seg) == 2:
            assert seg == [0, 1]


def test_empty_scene_is_zero_not_background():
    st = settings_for(_cam(), sh_degree=0, bg=(1.0, 1.0, 1.0))
    inp = dict(means3D=torch.zeros((0, 3)), opacities=torch.zeros((0, 1)), colors_precomp=torch.zeros((0, 3)),
               scales=torch.zeros((0, 3)), rotations=torch.zeros((0, 4)))
    run = oracle.forward(st, **inp)
    assert np.all(run.color == 0) and run.num_rendered == 0


@pytest.mark.parametrize("case", [
    dict(seed=0, sh_degree=3, include_feature=True),
    dict(seed=1, sh_degree=1, include_feature=True, bg=(0.3, 0.1, 0.7)),
    dict(seed=2, sh_degree=0, include_feature=False),
])
def test_forward_matches_dense_reference(case):
    st, inp = scene(P=250, W=48, H=40, scale_range=(0.03, 0.2), **case)
    run = oracle.forward(st, **inp)
    m2 = torch.zeros_like(inp["means3D"])
    color, lang, radii, ncon = torch_ref.rasterize(st, inp["means3D"], m2, inp["opacities"], shs=inp["shs"],
                                                   language_feature=inp["language_feature_precomp"],
                                                   scales=inp["scales"], rotations=inp["rotations"])
    np.testing.assert_array_equal(radii.numpy(), run.radii)
    np.testing.assert_array_equal(ncon.numpy(), run.get("n_contrib"))
    np.testing.assert_allclose(color.numpy(), run.color, atol=2e-5, rtol=0)
    np.testing.assert_allclose(lang.numpy(), run.language, atol=2e-5, rtol=0)


def _rel_err(a, b, floor):
    return np.max(np.abs(a - b) / (np.abs(b) + floor))


@pytest.mark.parametrize("case", [
    dict(seed=0, sh_degree=3, include_feature=True, bg=(0.0, 0.0, 0.0)),
    dict(seed=3, sh_degree=2, include_feature=True, bg=(0.5, 0.2, 0.9)),
    dict(seed=4, sh_degree=3, include_feature=False, bg=(1.0, 1.0, 1.0)),
])
def test_backward_matches_autograd_of_dense_reference(case):
    """Hand-derived oracle backward == torch.autograd through the dense formulation (float64)."""
    st, inp = scene(P=200, W=48, H=40, scale_range=(0.03, 0.2), **case)
    run = oracle.forward(st, **inp)
    gc, gl = grad_seed(40, 48, seed=7)
    ograd = run.backward(gc, gl)

    dt = torch.float64
    st64 = st._replace(bg=st.bg.to(dt), viewmatrix=st.viewmatrix.to(dt), projmatrix=st.projmatrix.to(dt),
                       campos=st.campos.to(dt))
    leaves = {k: v.to(dt).clone().requires_grad_(True) for k, v in inp.items()}
    m2 = torch.zeros_like(leaves["means3D"], requires_grad=True)
    color, lang, radii, ncon = torch_ref.rasterize(st64, leaves["means3D"], m2, leaves["opacities"],
                                                   shs=leaves["shs"],
                                                   language_feature=leaves["language_feature_precomp"],
                                                   scales=leaves["scales"], rotations=leaves["rotations"])
    np.testing.assert_array_equal(ncon.numpy(), run.get("n_contrib"))
    loss = (color * gc.to(dt)).sum() + (lang * gl.to(dt)).sum()
    loss.backward()
    checks = {
        "means3D": (leaves["means3D"].grad, ograd["means3D"]),
        "means2D": (m2.grad, ograd["means2D"]),
        "opacities": (leaves["opacities"].grad, ograd["opacities"]),
        "scales": (leaves["scales"].grad, ograd["scales"]),
        "rotations": (leaves["rotations"].grad, ograd["rotations"]),
        "shs": (leaves["shs"].grad, ograd["shs"]),
    }
    if case["include_feature"]:
        checks["language_feature_precomp"] = (leaves["language_feature_precomp"].grad,
                                              ograd["language_feature_precomp"])
    for name, (ref, ours) in checks.items():
        ref = ref.numpy()
        scale = np.max(np.abs(ref)) + 1e-12
        err = np.max(np.abs(ours - ref)) / scale
        assert err < 2e-4, (name, err)
