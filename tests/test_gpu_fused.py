"""Fused-activation path (include/lsr.h lsr_raw_flags) on the GPU.

Forward: bit-exact against the oracle fed with oracle.activate(raw) (kernels and oracle run
the same activation operation sequence).  Backward: the oracle's gradients w.r.t. the activated
tensors chained through oracle.activate_backward, with the tolerance of test_gpu_parity.  Then
render() with the fused path vs render() with LANGSPLAT_AMD_FUSED=0 (the reference's unfused
call on torch-activated inputs): images agree to the few-ulp activation differences and the
raw-parameter gradients agree within tolerance.
"""
import numpy as np
import pytest
import torch

from langsplat_amd import _native
from langsplat_amd.render import render
from langsplat_amd.synthetic import make_cameras, make_gaussians
from oracle import oracle
from tests.scenes import grad_seed, settings_for, to_device
from tests.test_gpu_parity import assert_grad_close, state

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _raw_scene(P, W, H, seed, sh_degree, include_feature=True, active_degree=None, scale_range=(0.03, 0.2)):
    g = make_gaussians(P, seed=seed, sh_degree=sh_degree, scale_range=scale_range)
    cam = make_cameras(1, W, H)[0]
    deg = sh_degree if active_degree is None else active_degree
    st = settings_for(cam, sh_degree=deg, include_feature=include_feature)
    return g, st


def _oracle_inputs(g, include_feature):
    a_op, a_sc, a_rot, a_lang = oracle.activate(oracle.RAW_ALL, g.opacity, g.scaling, g.rotation,
                                                g.language_feature)
    shs = torch.cat((g.features_dc, g.features_rest), dim=1)
    inp = dict(means3D=g.xyz.clone(), opacities=torch.from_numpy(a_op), scales=torch.from_numpy(a_sc),
               rotations=torch.from_numpy(a_rot), shs=shs.contiguous())
    if include_feature:
        inp["language_feature_precomp"] = torch.from_numpy(a_lang)
    return inp


FUSED_CASES = [
    dict(P=400, W=64, H=48, seed=0, sh_degree=3),
    dict(P=500, W=67, H=45, seed=1, sh_degree=3, active_degree=1),
    dict(P=300, W=48, H=40, seed=2, sh_degree=0),
    dict(P=600, W=80, H=64, seed=3, sh_degree=2, include_feature=False),
    # last block of 117 Gaussians: 5265 rest floats, a float4 run plus a 1-float tail (LDS-DMA staging)
    dict(P=501, W=64, H=48, seed=5, sh_degree=3),
    # _features_rest not 16-B aligned: the register-staged path
    dict(P=450, W=64, H=48, seed=6, sh_degree=3, misaligned=True),
]


@pytest.mark.parametrize("case", FUSED_CASES)
def test_fused_forward_bit_exact_and_backward(case):
    case = dict(case)
    misaligned = case.pop("misaligned", False)
    inc = case.get("include_feature", True)
    g, st = _raw_scene(**case)
    P, W, H = case["P"], case["W"], case["H"]
    inp = _oracle_inputs(g, inc)
    run = oracle.forward(st, **inp)
    std, _ = to_device(st, {}, DEV)
    gd = g.to(DEV)
    raw = _native.RAW_OPACITY | _native.RAW_SCALES | _native.RAW_ROTATIONS | (_native.RAW_LANGUAGE if inc else 0)
    rest = gd.features_rest.contiguous() if gd.features_rest.shape[1] > 0 else None
    if misaligned:
        buf = torch.empty(rest.numel() + 1, device=DEV)
        rest = buf[1:].view(rest.shape).copy_(rest)
        assert rest.data_ptr() % 16 != 0
    out = _native.rasterize_gaussians(std, gd.xyz, gd.features_dc.contiguous(), None,
                                      gd.language_feature if inc else None, gd.opacity, gd.scaling, gd.rotation,
                                      None, raw=raw, shs_rest=rest)
    nr, color, lang, radii, geom, binning, image = out
    assert nr == run.num_rendered
    np.testing.assert_array_equal(radii.cpu().numpy(), run.radii)
    np.testing.assert_array_equal(color.cpu().numpy(), run.color)
    np.testing.assert_array_equal(lang.cpu().numpy(), run.language)
    s = state(out, P, W, H)
    np.testing.assert_array_equal(s["n_contrib"], run.get("n_contrib"))
    np.testing.assert_array_equal(s["point_list"], run.get("point_list"))

    gc, gl = grad_seed(H, W, seed=4)
    ref = run.backward(gc, gl if inc else None)
    gr = _native.rasterize_gaussians_backward(
        std, gd.xyz, gd.features_dc.contiguous(), None, gd.language_feature if inc else None, gd.scaling,
        gd.rotation, None, radii, gc.to(DEV), gl.to(DEV) if inc else None, nr, geom, binning, image, raw=raw,
        shs_rest=rest, opacities=gd.opacity)
    torch.cuda.synchronize()
    d_op, d_sc, d_rot, d_lang = oracle.activate_backward(
        oracle.RAW_ALL if inc else oracle.RAW_ALL & ~oracle.RAW_LANGUAGE,
        (g.opacity, g.scaling, g.rotation, g.language_feature),
        (ref["opacities"], ref["scales"], ref["rotations"],
         ref.get("language_feature_precomp", np.zeros((P, 3), np.float32))))
    assert_grad_close("opacity_raw", gr["opacities"].cpu().numpy(), d_op)
    assert_grad_close("scaling_raw", gr["scales"].cpu().numpy(), d_sc)
    assert_grad_close("rotation_raw", gr["rotations"].cpu().numpy(), d_rot)
    if inc:
        assert_grad_close("language_raw", gr["language_feature_precomp"].cpu().numpy(), d_lang)
    assert_grad_close("means2D", gr["means2D"].cpu().numpy(), ref["means2D"])
    assert_grad_close("means3D", gr["means3D"].cpu().numpy(), ref["means3D"])
    assert_grad_close("features_dc", gr["shs"].cpu().numpy(), ref["shs"][:, :1])
    if rest is not None:
        assert_grad_close("features_rest", gr["shs_rest"].cpu().numpy(), ref["shs"][:, 1:])


class _Model:
    """GaussianModel's raw parameters + default activations (scene/gaussian_model.py:33-41)."""

    def __init__(self, g, device):
        self.max_sh_degree = self.active_sh_degree = g.max_sh_degree
        self.scaling_activation = torch.exp
        self.opacity_activation = torch.sigmoid
        self.rotation_activation = torch.nn.functional.normalize
        for n in ("xyz", "features_dc", "features_rest", "scaling", "rotation", "opacity", "language_feature"):
            setattr(self, "_" + n, getattr(g, n).to(device).clone().requires_grad_(True))

    get_xyz = property(lambda s: s._xyz)
    get_scaling = property(lambda s: torch.exp(s._scaling))
    get_rotation = property(lambda s: torch.nn.functional.normalize(s._rotation))
    get_opacity = property(lambda s: torch.sigmoid(s._opacity))
    get_features = property(lambda s: torch.cat((s._features_dc, s._features_rest), dim=1))
    get_language_feature = property(lambda s: s._language_feature)


class _Pipe:
    convert_SHs_python = False
    compute_cov3D_python = False
    debug = False


class _Opt:
    include_feature = True


def _render_grads(g, cam, fused, monkeypatch, gc, gl):
    monkeypatch.setenv("LANGSPLAT_AMD_FUSED", "1" if fused else "0")
    m = _Model(g, DEV)
    pkg = render(cam, m, _Pipe, torch.zeros(3, device=DEV), _Opt)
    ((pkg["render"] * gc).sum() + (pkg["language_feature_image"] * gl).sum()).backward()
    grads = {n: getattr(m, "_" + n).grad.detach().cpu().numpy()
             for n in ("xyz", "features_dc", "features_rest", "scaling", "rotation", "opacity", "language_feature")}
    grads["viewspace"] = pkg["viewspace_points"].grad.detach().cpu().numpy()
    # the fused path's visibility_filter comes from the preprocess kernel: same as radii > 0
    assert pkg["visibility_filter"].dtype == torch.bool
    assert torch.equal(pkg["visibility_filter"], pkg["radii"] > 0)
    return pkg["render"].detach(), pkg["language_feature_image"].detach(), pkg["radii"], grads


def test_render_fused_matches_unfused(monkeypatch):
    W, H = 96, 64
    g = make_gaussians(1500, seed=8, scale_range=(0.03, 0.2))
    cam = make_cameras(1, W, H, device=DEV)[0]
    gc, gl = (t.to(DEV) for t in grad_seed(H, W, seed=6))
    c0, l0, r0, g0 = _render_grads(g, cam, False, monkeypatch, gc, gl)
    c1, l1, r1, g1 = _render_grads(g, cam, True, monkeypatch, gc, gl)
    assert torch.equal(r0, r1)
    # torch's GPU sigmoid/exp/normalize and the restatement differ by a few ulp
    torch.testing.assert_close(c1, c0, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(l1, l0, rtol=1e-5, atol=1e-6)
    for k in g0:
        assert_grad_close(k, g1[k], g0[k])


@pytest.mark.parametrize("fused,colour", [(False, False), (True, False), (True, True)])
def test_language_step_skips_geometry_gradients(fused, colour, monkeypatch):
    """LangSplat's language step freezes every geometry parameter (scene/gaussian_model.py:203-217):
    the backward then computes only dL/dmeans2D and dL/dlanguage (include/lsr.h, geometry outputs
    all NULL) and must give what the full backward gives for those two (up to the order of the
    render backward's float atomics, which differs from run to run)."""
    W, H = 96, 64
    g = make_gaussians(1500, seed=9, scale_range=(0.03, 0.2))
    cam = make_cameras(1, W, H, device=DEV)[0]
    gc, gl = (t.to(DEV) for t in grad_seed(H, W, seed=12))
    monkeypatch.setenv("LANGSPLAT_AMD_FUSED", "1" if fused else "0")
    out = {}
    for force in (True, False):
        monkeypatch.setattr(_native, "FORCE_GEOMETRY_GRADS", force)
        m = _Model(g, DEV)
        for n in ("xyz", "features_dc", "features_rest", "scaling", "rotation", "opacity"):
            getattr(m, "_" + n).requires_grad_(False)
        pkg = render(cam, m, _Pipe, torch.zeros(3, device=DEV), _Opt)
        loss = (pkg["language_feature_image"] * gl).sum()
        if colour:  # the colour image in the loss too: the 12-value backward without geometry
            loss = loss + (pkg["render"] * gc).sum()
        loss.backward()
        out[force] = (m._language_feature.grad.detach().clone(), pkg["viewspace_points"].grad.detach().clone())
    for k in range(2):
        assert_grad_close(f"out{k}", out[False][k].cpu().numpy(), out[True][k].cpu().numpy())
    assert out[False][0].abs().sum() > 0


def _language_step(g, cam, gt, mask, fused_loss, monkeypatch, extra=None, geometry_frozen=True, colour_extra=None):
    """One language-feature train step (train.py:76-104): render, Ll1, backward.  colour_extra: the
    colour image also feeds a loss term (sum of image * colour_extra)."""
    monkeypatch.setenv("LANGSPLAT_AMD_FUSED", "1")
    m = _Model(g, DEV)
    if geometry_frozen:
        for n in ("xyz", "features_dc", "features_rest", "scaling", "rotation", "opacity"):
            getattr(m, "_" + n).requires_grad_(False)
    if fused_loss:
        pkg = render(cam, m, _Pipe, torch.zeros(3, device=DEV), _Opt, language_target=(gt, mask))
        loss = pkg["language_l1"]
    else:
        pkg = render(cam, m, _Pipe, torch.zeros(3, device=DEV), _Opt)
        loss = torch.abs(pkg["language_feature_image"] * mask - gt * mask).mean()
    total = loss if extra is None else loss + (pkg["language_feature_image"] * extra).sum()
    if colour_extra is not None:
        total = total + (pkg["render"] * colour_extra).sum()
    total.backward()
    grads = {"language_feature": m._language_feature.grad.detach().cpu().numpy(),
             "viewspace": pkg["viewspace_points"].grad.detach().cpu().numpy()}
    if not geometry_frozen:
        for n in ("xyz", "opacity", "scaling", "rotation", "features_dc"):
            grads[n] = getattr(m, "_" + n).grad.detach().cpu().numpy()
    return loss.detach(), pkg["language_feature_image"].detach(), grads


@pytest.mark.parametrize("W,H,extra,frozen", [(96, 64, False, True), (67, 45, True, True), (80, 48, False, False)])
def test_fused_language_loss_matches_torch_loss(W, H, extra, frozen, monkeypatch):
    """render(..., language_target=(gt, mask))["language_l1"] (loss inside the compositing kernel,
    its gradient folded into the replay's per-pixel seed) vs the same step with the loss as torch
    ops on the returned image (train.py:98): same image, loss within summation-order rounding,
    gradients within the parity tolerance (the render backward's float atomics differ run to run).
    extra: the language image also feeds a second loss term (the two gradients add)."""
    # P = 1503 in the odd-sized case: the gradient epilogue's four-per-thread form ends in a ragged tail
    g = make_gaussians(1500 + (W % 4), seed=10, scale_range=(0.03, 0.2))
    cam = make_cameras(1, W, H, device=DEV)[0]
    gen = torch.Generator().manual_seed(W)
    gt = torch.nn.functional.normalize(torch.randn((3, H, W), generator=gen), dim=0).to(DEV)
    mask = (torch.rand((1, H, W), generator=gen) < 0.8).to(DEV)
    ex = (torch.randn((3, H, W), generator=gen) / (3 * H * W)).to(DEV) if extra else None
    l0, img0, g0 = _language_step(g, cam, gt, mask, False, monkeypatch, ex, frozen)
    l1, img1, g1 = _language_step(g, cam, gt, mask, True, monkeypatch, ex, frozen)
    assert torch.equal(img0, img1)
    torch.testing.assert_close(l1, l0, rtol=2e-6, atol=0)
    for k in g0:
        assert_grad_close(k, g1[k], g0[k])
    assert np.abs(g1["language_feature"]).sum() > 0


@pytest.mark.parametrize("colour,frozen", [(False, True), (True, True), (True, False)])
def test_language_step_without_colour_state(colour, frozen, monkeypatch):
    """With language_target the forward is told no colour gradient follows (include/lsr.h
    LSR_FWD_NO_COLOR_GRAD): its split-replay states hold T and the feature sums only.  On a dense
    scene whose tiles composite past entries 256 / 512 / 768 (split replay active) the language step
    matches the unfused-loss step, whose forward keeps the colour sums.  colour: the colour image is
    in the loss too, so the backward rasterizes again with the colour sums (rasterizer.py) -- still
    the same gradients, geometry frozen or not."""
    W, H = 96, 80
    g = make_gaussians(40000, seed=21, scale_range=(0.02, 0.12))
    cam = make_cameras(1, W, H, device=DEV)[0]
    gen = torch.Generator().manual_seed(5)
    gt = torch.nn.functional.normalize(torch.randn((3, H, W), generator=gen), dim=0).to(DEV)
    mask = (torch.rand((1, H, W), generator=gen) < 0.8).to(DEV)
    cex = (torch.randn((3, H, W), generator=gen) / (3 * H * W)).to(DEV) if colour else None
    l0, img0, g0 = _language_step(g, cam, gt, mask, False, monkeypatch, None, frozen, cex)
    l1, img1, g1 = _language_step(g, cam, gt, mask, True, monkeypatch, None, frozen, cex)
    assert torch.equal(img0, img1)
    torch.testing.assert_close(l1, l0, rtol=2e-6, atol=0)
    for k in g0:
        assert_grad_close(k, g1[k], g0[k])
    assert np.abs(g1["viewspace"]).sum() > 0


def test_fused_language_loss_empty_scene(monkeypatch):
    """P = 0: the language image is all zeros; the loss is mean |0 - gt m|."""
    W, H = 40, 24
    g = make_gaussians(0, seed=0)
    cam = make_cameras(1, W, H, device=DEV)[0]
    gen = torch.Generator().manual_seed(1)
    gt = torch.randn((3, H, W), generator=gen).to(DEV)
    mask = (torch.rand((1, H, W), generator=gen) < 0.5).to(DEV)
    monkeypatch.setenv("LANGSPLAT_AMD_FUSED", "1")
    m = _Model(g, DEV)
    loss = render(cam, m, _Pipe, torch.zeros(3, device=DEV), _Opt, language_target=(gt, mask))["language_l1"]
    ref = torch.abs(torch.zeros_like(gt) * mask - gt * mask).mean()
    torch.testing.assert_close(loss, ref, rtol=2e-6, atol=0)


@pytest.mark.parametrize("fused_loss", [False, True])
def test_second_backward_clears_its_own_records(fused_loss, monkeypatch):
    """The forward clears the language step's gradient records inside its compositing kernel and
    the first backward uses them as they are (include/lsr.h LSR_FWD_ZERO_GRAD_RECORDS); a second
    backward over the same graph (retain_graph) must clear its own: same gradients both times."""
    W, H = 96, 64
    g = make_gaussians(1500, seed=13, scale_range=(0.03, 0.2))
    cam = make_cameras(1, W, H, device=DEV)[0]
    gen = torch.Generator().manual_seed(2)
    gt = torch.nn.functional.normalize(torch.randn((3, H, W), generator=gen), dim=0).to(DEV)
    mask = (torch.rand((1, H, W), generator=gen) < 0.8).to(DEV)
    monkeypatch.setenv("LANGSPLAT_AMD_FUSED", "1")
    m = _Model(g, DEV)
    for n in ("xyz", "features_dc", "features_rest", "scaling", "rotation", "opacity"):
        getattr(m, "_" + n).requires_grad_(False)
    if fused_loss:
        loss = render(cam, m, _Pipe, torch.zeros(3, device=DEV), _Opt, language_target=(gt, mask))["language_l1"]
    else:
        img = render(cam, m, _Pipe, torch.zeros(3, device=DEV), _Opt)["language_feature_image"]
        loss = torch.abs(img * mask - gt * mask).mean()
    loss.backward(retain_graph=True)
    g1 = m._language_feature.grad.detach().clone()
    m._language_feature.grad = None
    loss.backward()
    g2 = m._language_feature.grad.detach().clone()
    assert g1.abs().sum() > 0
    assert_grad_close("second backward", g2.cpu().numpy(), g1.cpu().numpy())


def test_fused_loss_wait_fallback_is_exact(monkeypatch):
    """The fused loss's last workgroup waits for every workgroup's word at most spin_limit polls
    (ADVICE r02); spin limit 0 sends every word not yet published through the fallback, which
    computes it from the inputs (the same pixels and operations as its workgroup: the oracle's
    compositing loop): the loss, the image and the gradients are bit-identical, and the stall is
    reported (lsr_debug_scan_stalls)."""
    lib = _native.load()
    W, H = 96, 64
    g = make_gaussians(1500, seed=10, scale_range=(0.03, 0.2))
    cam = make_cameras(1, W, H, device=DEV)[0]
    gen = torch.Generator().manual_seed(W)
    gt = torch.nn.functional.normalize(torch.randn((3, H, W), generator=gen), dim=0).to(DEV)
    mask = (torch.rand((1, H, W), generator=gen) < 0.8).to(DEV)
    l0, img0, g0 = _language_step(g, cam, gt, mask, True, monkeypatch)
    torch.cuda.synchronize()
    lib.lsr_debug_scan_stalls()  # clear
    old = lib.lsr_debug_set_spin_limit(0)
    try:
        l1, img1, g1 = _language_step(g, cam, gt, mask, True, monkeypatch)
        torch.cuda.synchronize()
        assert lib.lsr_debug_scan_stalls() == 1
    finally:
        lib.lsr_debug_set_spin_limit(old)
    assert torch.equal(l0, l1) and torch.equal(img0, img1)
    for k in g0:
        assert_grad_close(k, g1[k], g0[k])
