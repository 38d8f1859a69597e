"""The RGB stage's captured step across the model changes train.py makes between iterations (VERDICT r04
item 2): oneupSHdegree (train.py:81-82, scene/gaussian_model.py:166-168) raises the active SH degree,
a kernel argument of the captured preprocess, and reset_opacity (train.py:132-133,
scene/gaussian_model.py:277-281 + 326-339) replaces the opacity tensor and zeroes its moments, in the
reference's order inside its iteration (backward, reset, optimizer step: the new tensor has no
gradient, so its step count falls one behind the other groups').  GraphedStep(model=, optimizer=)
keys its capture on both (graph.capture_key) and re-captures at the next replay; the captured Adam
carries the per-parameter step offsets (include/lsr.h lsr_adam_multi, ABI 14).  The run must equal
the same loop done eagerly."""
import pytest
import torch

from langsplat_amd.densify import Densifier
from langsplat_amd.graph import GraphedStep
from langsplat_amd.optim import Adam
from langsplat_amd.render import render
from langsplat_amd.synthetic import make_cameras, make_gaussians
from tests.test_gpu_captured_forms import assert_close_mostly
from tests.test_gpu_fused import _Model, _Pipe

pytestmark = pytest.mark.gpu
DEV = "cuda"
ATTRS = {"xyz": "_xyz", "f_dc": "_features_dc", "f_rest": "_features_rest", "opacity": "_opacity",
         "scaling": "_scaling", "rotation": "_rotation"}


class _OptRGB:
    include_feature = False


def _rgb(g):
    m = _Model(g, DEV)
    m._language_feature.requires_grad_(False)
    m.active_sh_degree = 0  # train.py starts at degree 0 and raises it every 1000 iterations
    lr = {"xyz": 1.6e-4, "f_dc": 2.5e-3, "f_rest": 2.5e-3 / 20, "opacity": 0.05, "scaling": 5e-3, "rotation": 1e-3}
    # eps 1e-8 (not 1e-15): see tests/test_gpu_captured_forms.py _adam
    opt = Adam([{"params": [getattr(m, a)], "lr": lr[n], "name": n} for n, a in ATTRS.items()], lr=0.0, eps=1e-8)
    return m, opt


def _loss(m, cam, gt):
    pkg = render(cam, m, _Pipe, torch.zeros(3, device=DEV), _OptRGB)
    return torch.abs(pkg["render"] - gt).mean()


# the iterations: (SH degree bump before it, reset_opacity inside it)
SCHEDULE = [(False, False), (True, False), (False, False), (False, True), (True, False), (False, False),
            (True, False)]


def test_captured_rgb_step_across_sh_bumps_and_reset_opacity():
    P, W, H = 30000, 320, 240
    g = make_gaussians(P, seed=21, scale_range=(0.005, 0.05))
    cam = make_cameras(8, W, H, device=DEV)[2]
    gt = torch.rand((3, H, W), generator=torch.Generator().manual_seed(3)).to(DEV)
    runs = {}
    for form in ("eager", "graph"):
        m, opt = _rgb(g)

        def step():  # one view throughout (a captured step renders the view it was captured with)
            loss = _loss(m, cam, gt)
            loss.backward()
            return loss
        gs = None
        losses, degrees = [], []
        for k, (bump, reset) in enumerate(SCHEDULE):
            if bump:
                m.active_sh_degree = min(m.active_sh_degree + 1, m.max_sh_degree)  # oneupSHdegree
            degrees.append(m.active_sh_degree)
            if form == "eager" or reset:
                # the reference's iteration: backward, [reset_opacity], optimizer step, zero_grad
                if gs is not None:
                    gs.sync()
                opt.zero_grad(set_to_none=True)  # the graph's own .grad tensors are not accumulated into
                loss = step()
                if reset:
                    Densifier(m, opt).reset_opacity()
                opt.step()
                opt.zero_grad(set_to_none=True)
                losses.append(loss.detach().clone())
                del loss
            else:
                if gs is None:
                    gs = GraphedStep(step, [getattr(m, a) for a in ATTRS.values()], optimizer=opt, model=m)
                losses.append(gs.replay().clone())
        if gs is not None:
            torch.cuda.synchronize()
            assert gs.check()
            gs.sync()
        torch.cuda.synchronize()
        runs[form] = (torch.stack(losses), {n: getattr(m, a).detach().clone() for n, a in ATTRS.items()},
                      {n: int(opt.state[getattr(m, a)]["step"].item()) for n, a in ATTRS.items()},
                      gs.captures if gs is not None else 0, degrees)
    (le, pe, se, _, de), (lg, pg_, sg, caps, dg) = runs["eager"], runs["graph"]
    assert de == dg == [0, 1, 1, 1, 2, 2, 3]
    # the opacity group skipped the reset iteration's step: its count lags one behind
    assert se == sg and se["opacity"] == se["xyz"] - 1 == len(SCHEDULE) - 1
    # captures: the first, then one per bump or reset that a replay followed
    assert caps == 4
    torch.testing.assert_close(lg, le, rtol=1e-5, atol=0)
    for n in ATTRS:
        assert_close_mostly(n, pg_[n], pe[n], rtol=1e-5, atol=1e-6, outliers=1e-4)
