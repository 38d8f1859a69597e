"""Capacity mode (include/lsr.h lsr_forward_args.capacity_*) and the captured train step
(langsplat_amd.graph.GraphedStep).

Capacity mode sizes the binning from caller capacities and never waits for the device: its outputs
must be bit-identical to the eager forward's (images, radii, per-tile ranges and order, final T,
contributor counts), its backward identical too, and a view over capacity must be flagged and left
un-rasterized (background, no out-of-bounds writes).  The captured step must reproduce the eager
language step (train.py:92-104) loss and gradients on every replay.
"""
import numpy as np
import pytest
import torch

from langsplat_amd import _native
from langsplat_amd.graph import GraphedStep
from langsplat_amd.render import render
from langsplat_amd.synthetic import make_cameras, make_gaussians
from tests.scenes import grad_seed, scene, to_device
from tests.test_gpu_fused import _Model, _Opt, _Pipe
from tests.test_gpu_parity import assert_grad_close, state

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _forward(st, ind, cap=None, flags=0):
    args = (ind["means3D"], ind["shs"], None, ind["language_feature_precomp"], ind["opacities"], ind["scales"],
            ind["rotations"], None)
    if cap is None:
        out = _native.rasterize_gaussians(st, *args, flags=flags)
    else:
        with cap:
            out = _native.rasterize_gaussians(st, *args, flags=flags)
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("P,W,H", [(3000, 160, 120), (20000, 640, 360)])
def test_capacity_mode_matches_eager(P, W, H):
    st, inp = scene(P=P, W=W, H=H, seed=4, scale_range=(0.02, 0.15))
    std, ind = to_device(st, inp, DEV)
    eager = _forward(std, ind)
    R, E = _native.LAST_COUNTS[(P, W, H)]
    assert R == eager[0] and E > 0
    ovf = torch.full((), 7, dtype=torch.int32, device=DEV)
    capd = _forward(std, ind, _native.capacity(R + 100, E + 10, ovf))
    assert int(ovf.item()) == 0
    assert capd[0] == R + 100  # the layout key lsr_backward needs
    for a, b in zip(eager[1:4], capd[1:4]):
        assert torch.equal(a, b)
    se, sc = state(eager, P, W, H), state(capd, P, W, H)
    np.testing.assert_array_equal(se["ranges"], sc["ranges"])
    np.testing.assert_array_equal(se["final_T"], sc["final_T"])
    np.testing.assert_array_equal(se["n_contrib"], sc["n_contrib"])
    np.testing.assert_array_equal(se["point_list"], sc["point_list"][:R])
    # exact capacities fit too
    capx = _forward(std, ind, _native.capacity(R, E, ovf))
    assert int(ovf.item()) == 0 and torch.equal(capx[1], eager[1])
    # the backward over the capacity-mode state
    gc, gl = grad_seed(H, W, seed=5)
    bw = lambda out: _native.rasterize_gaussians_backward(  # noqa: E731
        std, ind["means3D"], ind["shs"], None, ind["language_feature_precomp"], ind["scales"], ind["rotations"], None,
        out[3], gc.to(DEV), gl.to(DEV), out[0], out[4], out[5], out[6])
    ge, gcap = bw(eager), bw(capd)
    for k in ("means2D", "opacities", "means3D", "language_feature_precomp", "shs", "scales", "rotations"):
        assert_grad_close(k, gcap[k].cpu().numpy(), ge[k].cpu().numpy())


@pytest.mark.parametrize("short", ["rendered", "entries"])
def test_capacity_overflow_is_flagged_and_safe(short):
    """A view over capacity: flagged, background image, zero contributors -- and the next forward
    with room is exact again (nothing was written out of bounds)."""
    P, W, H = 4000, 128, 96
    st, inp = scene(P=P, W=W, H=H, seed=6, scale_range=(0.03, 0.2), bg=(0.25, 0.5, 0.75))
    std, ind = to_device(st, inp, DEV)
    eager = _forward(std, ind)
    R, E = _native.LAST_COUNTS[(P, W, H)]
    ovf = torch.zeros((), dtype=torch.int32, device=DEV)
    cap = _native.capacity(R // 2, E, ovf) if short == "rendered" else _native.capacity(R, E // 2, ovf)
    out = _forward(std, ind, cap)
    assert ovf.view(torch.float32).item() == 1.0  # the bits of 1.0f (include/lsr.h)
    bg = torch.tensor([0.25, 0.5, 0.75], device=DEV).view(3, 1, 1).expand(3, H, W)
    assert torch.equal(out[1], bg) and not out[2].any()
    assert not state(out, P, W, H)["n_contrib"].any()
    ok = _forward(std, ind, _native.capacity(R, E, ovf))
    assert int(ovf.item()) == 0 and torch.equal(ok[1], eager[1]) and torch.equal(ok[2], eager[2])


def _language_setup(W=160, H=120, P=6000):
    g = make_gaussians(P, seed=17, scale_range=(0.02, 0.15))
    cam = make_cameras(1, W, H, device=DEV)[0]
    gen = torch.Generator().manual_seed(3)
    gt = torch.nn.functional.normalize(torch.randn((3, H, W), generator=gen), dim=0).to(DEV)
    mask = (torch.rand((1, H, W), generator=gen) < 0.9).to(DEV)
    m = _Model(g, DEV)
    for n in ("xyz", "features_dc", "features_rest", "scaling", "rotation", "opacity"):
        getattr(m, "_" + n).requires_grad_(False)
    bg = torch.zeros(3, device=DEV)

    def forward():
        return render(cam, m, _Pipe, bg, _Opt, language_target=(gt, mask))["language_l1"]

    def step():
        loss = forward()
        loss.backward()
        return loss
    step.forward = forward
    return m, step


def test_graphed_language_step_matches_eager(monkeypatch):
    monkeypatch.setenv("LANGSPLAT_AMD_FUSED", "1")
    m, step = _language_setup()
    m._language_feature.grad = None
    loss0 = step().detach().clone()
    g0 = m._language_feature.grad.detach().clone()
    gs = GraphedStep(step, [m._language_feature])
    for it in range(3):
        loss = gs.replay()
        torch.cuda.synchronize()
        assert gs.check()
        torch.testing.assert_close(loss, loss0, rtol=0, atol=0)
        assert_grad_close(f"replay {it}", m._language_feature.grad.cpu().numpy(), g0.cpu().numpy())
    assert gs.captures == 1


def test_graphed_step_recaptures_on_overflow(monkeypatch):
    """Capacities from the warm-up view; the parameters then change so that the view needs more
    tile instances than captured: check() reports it once and re-captures; the next replay fits and
    matches the eager step."""
    monkeypatch.setenv("LANGSPLAT_AMD_FUSED", "1")
    m, step = _language_setup(P=3000)
    gs = GraphedStep(step, [m._language_feature], headroom=1.0)
    gs.capture()
    gs.rendered_at_capture = gs.rendered
    with torch.no_grad():
        m._scaling.add_(0.7)  # twice the size: many more tile instances
    gs.replay()
    assert not gs.check() and gs.captures == 2 and gs.rendered > gs.rendered_at_capture
    loss = gs.replay().detach().clone()
    assert gs.check()
    g1 = m._language_feature.grad.detach().clone()
    m._language_feature.grad = None
    loss_e = step()
    torch.testing.assert_close(loss, loss_e.detach(), rtol=0, atol=0)
    assert_grad_close("after recapture", g1.cpu().numpy(), m._language_feature.grad.cpu().numpy())


def test_graphed_step_with_adam_matches_eager_steps(monkeypatch):
    """Adam captured with the step (its step count on the device): K replays give the parameters and
    moments of K eager steps (to float rounding), and sync() brings the step count back to the host."""
    from langsplat_amd.optim import Adam
    monkeypatch.setenv("LANGSPLAT_AMD_FUSED", "1")
    runs = {}
    for mode in ("eager", "graph"):
        m, step = _language_setup(P=4000)
        opt = Adam([{"params": [m._language_feature], "lr": 0.01, "name": "language_feature"}], lr=0.0, eps=1e-15)
        if mode == "eager":
            for _ in range(5):  # five replays (GraphedStep's warm-up steps do not step the optimizer)
                m._language_feature.grad = None
                step()
                opt.step()
        else:
            gs = GraphedStep(step, [m._language_feature], optimizer=opt)
            for _ in range(5):
                gs.replay()
            assert gs.check()
            gs.sync()
        torch.cuda.synchronize()
        st = opt.state[m._language_feature]
        runs[mode] = (m._language_feature.detach().clone(), st["exp_avg"].clone(), st["exp_avg_sq"].clone(),
                      int(st["step"].item()))
    (pe, me, ve, se), (pg, mg, vg, sg) = runs["eager"], runs["graph"]
    assert se == sg == 5
    torch.testing.assert_close(pg, pe, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(mg, me, rtol=1e-4, atol=1e-9)
    torch.testing.assert_close(vg, ve, rtol=1e-4, atol=1e-12)


def _depth_scene(P, W, H, wide, seed):
    """Gaussians in front of camera 0 (view depth = z + 4) over a wide (0.3..80) or narrow depth range."""
    import math
    g = torch.Generator().manual_seed(seed)
    if wide:
        d = torch.exp(torch.rand(P, generator=g) * (math.log(80.0) - math.log(0.3)) + math.log(0.3))
    else:
        d = 4.0 + torch.rand(P, generator=g) * 1e-3
    u, v = torch.rand(P, generator=g) * 2 - 1, torch.rand(P, generator=g) * 2 - 1
    means = torch.stack([u * d * 0.4, v * d * 0.3, d - 4.0], 1)
    from tests.scenes import settings_for
    st = settings_for(make_cameras(1, W, H)[0], sh_degree=3)
    inp = dict(means3D=means, opacities=torch.rand((P, 1), generator=g) * 0.6 + 0.05,
               shs=torch.randn((P, 16, 3), generator=g) * 0.2,
               language_feature_precomp=torch.nn.functional.normalize(torch.randn((P, 3), generator=g)),
               scales=torch.full((P, 3), 0.02) * d[:, None] / 4.0,
               rotations=torch.nn.functional.normalize(torch.randn((P, 4), generator=g)))
    return to_device(st, inp, DEV)


def test_capacity_mode_lsd_depth_order(monkeypatch):
    """The LSD depth order (P > 4.2M, forced here by LSR_DEPTH_LSD=1) in capacity mode uses the pass
    count of the thread's last eager forward: exact when it suffices (also when it exceeds the view's
    need), flagged when the view's key range needs more passes, exact again after an eager forward of
    that view."""
    monkeypatch.setenv("LSR_DEPTH_LSD", "1")
    P, W, H = 3000, 96, 64
    narrow = _depth_scene(P, W, H, False, 41)
    wide = _depth_scene(P, W, H, True, 42)
    e_wide = _forward(*wide)
    Rw, Ew = _native.LAST_COUNTS[(P, W, H)]
    ovf = torch.zeros((), dtype=torch.int32, device=DEV)
    c_wide = _forward(*wide, cap=_native.capacity(Rw, Ew, ovf))
    assert int(ovf.item()) == 0 and torch.equal(c_wide[1], e_wide[1])
    np.testing.assert_array_equal(state(c_wide, P, W, H)["point_list"][:Rw], state(e_wide, P, W, H)["point_list"])
    # more passes than the view needs (the wide view's 4 for the narrow one's 2): the passes above its
    # key range see one digit and take the scatter's identity path -- the same order
    c_narrow = _forward(*narrow, cap=_native.capacity(400000, 400000, ovf))
    assert int(ovf.item()) == 0
    e_narrow = _forward(*narrow)  # the thread's last eager view now needs fewer passes
    Rn = _native.LAST_COUNTS[(P, W, H)][0]
    assert torch.equal(c_narrow[1], e_narrow[1]) and torch.equal(c_narrow[2], e_narrow[2])
    np.testing.assert_array_equal(state(c_narrow, P, W, H)["point_list"][:Rn], state(e_narrow, P, W, H)["point_list"])
    c2 = _forward(*wide, cap=_native.capacity(Rw, Ew, ovf))
    assert ovf.view(torch.float32).item() == 1.0 and not c2[2].any()
    _forward(*wide)
    c3 = _forward(*wide, cap=_native.capacity(Rw, Ew, ovf))
    assert int(ovf.item()) == 0 and torch.equal(c3[1], e_wide[1])
