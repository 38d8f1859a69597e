"""The captured step forms at the size they are benched at, over view sequences, and on overflow
(VERDICT r03 "next round" item 1).

bench.py's `value` comes from langsplat_amd.pipeline.PipelinedGraphStep (capacity mode, the forward
split in its geometry and composite halves, graphs on two streams).  Here, at full C3 (BASELINE.json
configs[2]) and C5 (configs[4], the 512-bucket MSD depth order; the LSD passes where a test sets
LSR_DEPTH_LSD=1):
  - the capacity-mode forward is bit-identical to the eager one and its backward matches it;
  - the benched pipelined form's first replay matches the oracle's language step (images bit for
    bit, loss, d(loss)/d(_language_feature)), and its later replays equal eager serial steps.
Over a rotating C4 view sequence (train.py:85-87 picks a random view every iteration), GraphedStep
and PipelinedGraphStep (2 and 3 buffer sets) load each view -- camera and language target -- into
their ViewSlots and reproduce the eager loop.  A view forced over capacity mid-sequence is a no-op
for the optimiser (parameters, moments and step count bit-unchanged across that replay: the view is
left out), check() reports it and the replays continue after a re-capture.

Tolerances: images and losses of the first step bit-exact / 2e-6 (the oracle); later steps carry
the backward's float-atomic rounding (its order varies between any two runs), so losses agree to
1e-5 relative and parameters / moments as in tests/test_gpu_pipeline.py, on all but 1e-5 of the
entries (an entry whose gradient cancels to ~0 can flip the sign of Adam's first update).
"""
import numpy as np
import pytest
import torch

from langsplat_amd import _native
from langsplat_amd.graph import GraphedStep, ViewSlot
from langsplat_amd.distributed import GradBucket
from langsplat_amd.optim import Adam
from langsplat_amd.pipeline import PipelinedGraphStep
from langsplat_amd.render import render
from langsplat_amd.synthetic import CONFIGS, activated_inputs, make_cameras, make_gaussians
from tests.scenes import settings_for
from tests.test_gpu_fused import _Model, _Opt, _Pipe
from tests.test_gpu_parity import assert_grad_close, state
from tests.test_gpu_timed_step import bench_target, oracle_language_step

pytestmark = pytest.mark.gpu
DEV = "cuda"
LR = 0.0025  # bench.py's language-feature lr (scene/gaussian_model.py:203-217 with the default args)


def _frozen_model(g):
    m = _Model(g, DEV)
    for n in ("xyz", "features_dc", "features_rest", "scaling", "rotation", "opacity"):
        getattr(m, "_" + n).requires_grad_(False)
    return m


def _adam(m, lr=LR):
    """The language step's Adam (scene/gaussian_model.py:217-229) with eps 1e-8 instead of 1e-15: with
    1e-15 a Gaussian whose gradient is float-atomic noise (~1e-12, an occluded one) moves by a full
    +-lr whose sign is that noise, so two runs of ANY form drift apart by ~1e-4 of the loss within a
    few steps (measured at C3).  1e-8 keeps such updates ~1e-4 lr while every gradient of a visible
    Gaussian (~1e-6) still takes a ~full-size step: the comparisons below then test the forms, not
    the noise.  (bench.py and the single-step oracle checks keep 1e-15.)"""
    return Adam([{"params": [m._language_feature], "lr": lr, "name": "language_feature"}], lr=0.0, eps=1e-8)


def _state(m, opt):
    st = opt.state[m._language_feature]
    return (m._language_feature.detach().clone(), st["exp_avg"].clone(), st["exp_avg_sq"].clone())


def assert_close_mostly(name, got, want, rtol, atol, outliers=1e-5):
    """|got - want| <= atol + rtol |want| on all but `outliers` of the entries."""
    got, want = got.double(), want.double()
    bad = (got - want).abs() > atol + rtol * want.abs()
    n = int(bad.sum().item())
    assert n <= outliers * bad.numel(), f"{name}: {n} / {bad.numel()} entries off " \
                                        f"(max |diff| {float((got - want).abs().max().item()):.3e})"


def assert_states_close(a, b, tag):
    for name, x, y, rtol, atol in (("param", a[0], b[0], 1e-5, 1e-6), ("exp_avg", a[1], b[1], 1e-4, 1e-9),
                                   ("exp_avg_sq", a[2], b[2], 1e-4, 1e-12)):
        assert_close_mostly(f"{tag} {name}", x, y, rtol, atol)


def _eager_step(m, opt, cam, gt, mask):
    loss = render(cam, m, _Pipe, torch.zeros(3, device=DEV), _Opt, language_target=(gt, mask))["language_l1"]
    loss.backward()
    opt.step()
    opt.zero_grad(set_to_none=True)
    return loss.detach().clone()


# ---- capacity mode at full size --------------------------------------------------------------------

@pytest.mark.parametrize("cfg", ["C3", "C5"])
def test_capacity_mode_matches_eager_full_size(cfg, monkeypatch):
    """The benched language step's forward (fused activations + fused loss, raw parameters) in
    capacity mode against the eager forward at full size: images, radii, loss, per-tile ranges and
    order, final T and contributor counts bit-identical; the language-step backward's gradients
    within the parity tolerance.  C5 (3M Gaussians) takes the 512-bucket MSD depth order."""
    monkeypatch.setenv("LANGSPLAT_AMD_FUSED", "1")
    c = CONFIGS[cfg]
    P, W, H = c["P"], c["width"], c["height"]
    g = make_gaussians(P, seed=0)
    cam = make_cameras(c["views"], W, H, device=DEV)[0]
    gt, mask = (t.to(DEV) for t in bench_target(H, W, 0))
    outs = []
    for mode in ("eager", "capacity"):
        m = _frozen_model(g)
        sb = _native.static_buffers()
        ov = torch.full((), 7, dtype=torch.int32, device=DEV)
        if mode == "eager":
            with sb:
                pkg = render(cam, m, _Pipe, torch.zeros(3, device=DEV), _Opt, language_target=(gt, mask))
            R, E = _native.LAST_COUNTS[(P, W, H)]
        else:
            with sb, _native.capacity(int(R * 1.125) + 1024, int(E * 1.125) + 1024, ov):
                pkg = render(cam, m, _Pipe, torch.zeros(3, device=DEV), _Opt, language_target=(gt, mask))
        pkg["language_l1"].backward()
        torch.cuda.synchronize()
        if mode == "capacity":
            assert int(ov.item()) == 0
        geom, binning, image = (sb.tensors[("scratch", k)] for k in (0, 1, 2))
        outs.append(dict(color=pkg["render"].detach().clone(), lang=pkg["language_feature_image"].detach().clone(),
                         radii=pkg["radii"].clone(), loss=pkg["language_l1"].detach().clone(),
                         grad=m._language_feature.grad.detach().cpu().numpy(),
                         vgrad=pkg["viewspace_points"].grad.detach().cpu().numpy(),
                         st=state((R, None, None, None, geom, binning, image), P, W, H)))
    e, cp = outs
    for k in ("color", "lang", "radii", "loss"):
        assert torch.equal(e[k], cp[k]), k
    for k in ("ranges", "final_T", "n_contrib"):
        np.testing.assert_array_equal(e["st"][k], cp["st"][k])
    np.testing.assert_array_equal(e["st"]["point_list"][:R], cp["st"]["point_list"][:R])
    assert_grad_close("language_feature (raw)", cp["grad"], e["grad"])
    assert_grad_close("viewspace_points", cp["vgrad"], e["vgrad"])


# ---- the benched form at the benched size ------------------------------------------------------------

def test_pipelined_graph_full_c3_matches_oracle_and_eager(monkeypatch):
    """bench.py's PipelinedGraphStep at C3: the first replay against oracle_language_step (images bit
    for bit, loss, the raw language-feature gradient), then K replays against K eager serial steps of
    the same view (losses, parameters, Adam moments, device step count)."""
    monkeypatch.setenv("LANGSPLAT_AMD_FUSED", "1")
    c = CONFIGS["C3"]
    P, W, H = c["P"], c["width"], c["height"]
    g = make_gaussians(P, seed=0)
    cam_cpu = make_cameras(1, W, H)[0]
    gt_cpu, mask_cpu = bench_target(H, W, 0)
    run, loss_ref, d_lang_ref, _ = oracle_language_step(g, cam_cpu, gt_cpu, mask_cpu)
    cam, gt, mask = cam_cpu.to(DEV), gt_cpu.to(DEV), mask_cpu.to(DEV)
    K = 4
    # eager serial steps
    me = _frozen_model(g)
    oe = _adam(me)
    eager_losses = [_eager_step(me, oe, cam, gt, mask) for _ in range(1 + K)]
    se = _state(me, oe)
    # the benched form
    mg = _frozen_model(g)
    og = _adam(mg)
    bg = torch.zeros(3, device=DEV)
    pg = PipelinedGraphStep(lambda: render(cam, mg, _Pipe, bg, _Opt, language_target=(gt, mask))["language_l1"],
                            [mg._language_feature], og).capture()
    assert pg.S == 3 and pg.fused  # bench.py's form: three buffer sets, the fused language-step tail
    first = pg.replay().clone()
    pg.synchronize()
    torch.cuda.synchronize()
    out = pg.sets[0].tensors
    np.testing.assert_array_equal(out[("out", "color")].detach().cpu().numpy(), run.color)
    np.testing.assert_array_equal(out[("out", "language")].detach().cpu().numpy(), run.language)
    np.testing.assert_array_equal(out[("out", "radii")].detach().cpu().numpy(), run.radii)
    assert abs(float(first.item()) - loss_ref) <= 2e-6 * loss_ref
    assert_grad_close("language_feature (raw), first replay", pg.last_grads()[0].detach().cpu().numpy(), d_lang_ref)
    losses = [first] + [pg.replay().clone() for _ in range(K)]
    pg.synchronize()
    torch.cuda.synchronize()
    assert pg.check() and pg.captures == 1
    pg.sync()
    assert int(og.state[mg._language_feature]["step"].item()) == 1 + K
    assert torch.equal(losses[0], eager_losses[0])
    torch.testing.assert_close(torch.stack(losses), torch.stack(eager_losses), rtol=1e-5, atol=0)
    assert_states_close(_state(mg, og), se, "C3 pipelined graph")


def test_graphed_step_full_c5_matches_eager(monkeypatch):
    """GraphedStep (one graph: render + loss + backward + Adam) at C5 with the depth order as LSD
    passes (LSR_DEPTH_LSD=1, the order above 4.2M Gaussians) and the pass count of the last eager
    forward: 3 replays equal 3 eager steps."""
    monkeypatch.setenv("LANGSPLAT_AMD_FUSED", "1")
    monkeypatch.setenv("LSR_DEPTH_LSD", "1")
    c = CONFIGS["C5"]
    P, W, H = c["P"], c["width"], c["height"]
    g = make_gaussians(P, seed=0)
    cam = make_cameras(c["views"], W, H, device=DEV)[0]
    gt, mask = (t.to(DEV) for t in bench_target(H, W, 0))
    K = 3
    me = _frozen_model(g)
    oe = _adam(me)
    eager_losses = [_eager_step(me, oe, cam, gt, mask) for _ in range(K)]
    se = _state(me, oe)
    del me, oe
    mg = _frozen_model(g)
    og = _adam(mg)
    bg = torch.zeros(3, device=DEV)

    def step():
        loss = render(cam, mg, _Pipe, bg, _Opt, language_target=(gt, mask))["language_l1"]
        loss.backward()
        return loss
    gs = GraphedStep(step, [mg._language_feature], optimizer=og).capture()
    losses = [gs.replay().clone() for _ in range(K)]
    torch.cuda.synchronize()
    assert gs.check() and gs.captures == 1
    gs.sync()
    assert int(og.state[mg._language_feature]["step"].item()) == K
    assert torch.equal(losses[0], eager_losses[0])
    torch.testing.assert_close(torch.stack(losses), torch.stack(eager_losses), rtol=1e-5, atol=0)
    assert_states_close(_state(mg, og), se, "C5 graph")


# ---- a rotating view sequence ------------------------------------------------------------------------

SEQ = [0, 3, 5, 1, 7, 2, 6, 4]


def _c4_views(seq=SEQ, radius=4.0, cfg="C4", P=None):
    c = CONFIGS[cfg]
    W, H = c["width"], c["height"]
    cams = make_cameras(8, W, H, radius=radius, device=DEV)
    views = []
    for v in seq:
        gt, mask = bench_target(H, W, v)
        views.append((cams[v], gt.to(DEV), mask.to(DEV)))
    return views


def _eager_sequence(g, views):
    m = _frozen_model(g)
    opt = _adam(m)
    R = E = 0
    losses = []
    for cam, gt, mask in views:
        losses.append(_eager_step(m, opt, cam, gt, mask))
        r, e = next(iter(_native.LAST_COUNTS.values()))
        R, E = max(R, r), max(E, e)
    torch.cuda.synchronize()
    return losses, _state(m, opt), (int(R * 1.05) + 1024, int(E * 1.05) + 1024)


def _slot_forward(m):
    bg = torch.zeros(3, device=DEV)
    return lambda slot: render(slot, m, _Pipe, bg, _Opt, language_target=slot.language_target)["language_l1"]


def test_graphed_step_over_a_view_sequence(monkeypatch):
    """GraphedStep with a ViewSlot: replay(view=...) loads each view's camera and target; the replays
    reproduce the eager loop over the same rotating C4 sequence."""
    monkeypatch.setenv("LANGSPLAT_AMD_FUSED", "1")
    g = make_gaussians(CONFIGS["C4"]["P"], seed=0)
    views = _c4_views()
    losses_e, se, (Rc, Ec) = _eager_sequence(g, views)
    m = _frozen_model(g)
    opt = _adam(m)
    slot = ViewSlot(*views[0])
    fwd = _slot_forward(m)

    def step():
        loss = fwd(slot)
        loss.backward()
        return loss
    gs = GraphedStep(step, [m._language_feature], optimizer=opt, view=slot).capture(Rc, Ec)
    losses = [gs.replay(view=v).clone() for v in views]
    torch.cuda.synchronize()
    assert gs.check() and gs.captures == 1
    gs.sync()
    assert int(opt.state[m._language_feature]["step"].item()) == len(views)
    assert torch.equal(losses[0], losses_e[0])
    torch.testing.assert_close(torch.stack(losses), torch.stack(losses_e), rtol=1e-5, atol=0)
    assert_states_close(_state(m, opt), se, "graph sequence")


@pytest.mark.parametrize("sets,wait,bucket", [(2, True, False), (3, True, False), (3, False, False),
                                              (3, True, "defer"), (2, True, "defer"), (3, True, "fill"),
                                              (3, True, "python"), (3, False, "python")])
def test_pipelined_graph_over_a_view_sequence(sets, wait, bucket, monkeypatch):
    """PipelinedGraphStep with one ViewSlot per buffer set: capture(views=the first S - 1 views),
    replay(next_view=the view S - 1 ahead); every replay composites its own view's geometry with its
    own target, and the sequence reproduces the eager loop.  wait=False (bench.py's form): no
    per-replay join with the caller's stream, the views loaded on the geometry stream; the last S
    losses (valid after synchronize()) and the final state reproduce the eager loop.  bucket (round
    6): the N > 1 structure on one process (a GradBucket, no process group: its all-reduce is a
    no-op) -- the backward and the update as two graphs, the update filling the next set's records
    (lsr_adam_fill_language), the first composite refilled from the parameter.  "defer" (the default
    since ABI 16): the backward leaves the language partials, the collective reduces them and ONE
    tail pass (lsr_language_tail) writes the gradients, steps and fills; "fill" (LSR_PG_DEFER=0): the
    epilogue in the backward, then lsr_adam_fill_language.  "python": no bucket, and every replay
    through torch's stream context and CUDAGraph.replay() instead of the native steady-state launch
    (lsr_graph_launch, LSR_PG_NATIVE_LAUNCH=0)."""
    import langsplat_amd.pipeline as pipeline_mod
    monkeypatch.setenv("LANGSPLAT_AMD_FUSED", "1")
    native = bucket != "python"
    monkeypatch.setattr(pipeline_mod, "_NATIVE_LAUNCH", native)
    bucket = False if bucket == "python" else bucket
    monkeypatch.setenv("LSR_PG_DEFER", "0" if bucket == "fill" else "1")
    g = make_gaussians(CONFIGS["C4"]["P"], seed=0)
    views = _c4_views()
    losses_e, se, (Rc, Ec) = _eager_sequence(g, views)
    m = _frozen_model(g)
    opt = _adam(m)
    slots = [ViewSlot(*views[0]) for _ in range(sets)]
    pg = PipelinedGraphStep(_slot_forward(m), [m._language_feature], opt, slots=slots,
                            bucket=GradBucket([m._language_feature]) if bucket else None)
    pg.capture(Rc, Ec, views=views[:sets - 1])
    assert pg.fill_after == bool(bucket) and (pg.g_adam[0] is not None) == bool(bucket)
    assert pg.defer == (bucket == "defer")
    L = sets - 1
    losses = []
    for k in range(len(views)):
        nxt = views[k + L] if k + L < len(views) else None
        if wait:
            losses.append(pg.replay(next_view=nxt).clone())
        else:
            losses.append(pg.replay(next_view=nxt, wait=False))
    pg.synchronize()
    torch.cuda.synchronize()
    if not wait:  # only the last S replays' static losses are still theirs
        losses = [t.clone() for t in losses[-sets:]]
        losses_e = losses_e[-sets:]
    assert pg.check() and pg.captures == 1
    # the steady-state replays of the N = 1 form went through the native launch (lsr_graph_launch)
    assert bool(pg._launchers) == (native and not bucket)
    pg.sync()
    assert int(opt.state[m._language_feature]["step"].item()) == len(views)
    if wait:
        assert torch.equal(losses[0], losses_e[0])
    torch.testing.assert_close(torch.stack(losses), torch.stack(losses_e), rtol=1e-5, atol=0)
    assert_states_close(_state(m, opt), se, f"pipelined graph sequence, {sets} sets, wait={wait}")


@pytest.mark.parametrize("rot,wait", [(2, True), (2, False), (4, False)])
def test_pipelined_graph_rotation_over_a_view_sequence(rot, wait, monkeypatch):
    """Rotation mode (R steps per stream-A graph over 2 R buffer sets): the 8-view C4 sequence
    (a multiple of R replays) reproduces the eager loop -- the last R losses after synchronize()
    and the final parameters, moments and step count."""
    monkeypatch.setenv("LANGSPLAT_AMD_FUSED", "1")
    g = make_gaussians(CONFIGS["C4"]["P"], seed=0)
    views = _c4_views()
    assert len(views) % rot == 0
    losses_e, se, (Rc, Ec) = _eager_sequence(g, views)
    m = _frozen_model(g)
    opt = _adam(m)
    S = 2 * rot
    slots = [ViewSlot(*views[0]) for _ in range(S)]
    pg = PipelinedGraphStep(_slot_forward(m), [m._language_feature], opt, slots=slots, rotation=rot)
    assert pg.S == S and pg.R == rot
    pg.capture(Rc, Ec, views=views[:S - 1])
    losses = []
    for k in range(len(views)):
        nxt = views[k + S - 1] if k + S - 1 < len(views) else None
        losses.append(pg.replay(next_view=nxt, wait=wait))
    pg.synchronize()
    torch.cuda.synchronize()
    losses = [t.clone() for t in losses[-rot:]]
    assert pg.check() and pg.captures == 1
    pg.sync()
    assert int(opt.state[m._language_feature]["step"].item()) == len(views)
    torch.testing.assert_close(torch.stack(losses), torch.stack(losses_e[-rot:]), rtol=1e-5, atol=0)
    assert_states_close(_state(m, opt), se, f"pipelined graph rotation {rot}, wait={wait}")


# ---- a view over capacity mid-sequence ---------------------------------------------------------------

def _overflow_views(W=320, H=240):
    """Five views of a small scene; the third is a camera pulled in close (same field of view), with
    several times the tile instances of the others."""
    far = make_cameras(8, W, H, radius=4.0, device=DEV)
    near = make_cameras(8, W, H, radius=1.6, device=DEV)
    cams = [far[0], far[2], near[1], far[5], far[3]]
    out = []
    for i, cam in enumerate(cams):
        gt, mask = bench_target(H, W, i)
        out.append((cam, gt.to(DEV), mask.to(DEV)))
    return out


def _snap(m, opt):
    st = opt.state[m._language_feature]
    return (m._language_feature.detach().clone(), st["exp_avg"].clone(), st["exp_avg_sq"].clone(),
            int(opt._step_dev[0].item()))


def _assert_bit_equal(a, b):
    for x, y in zip(a[:3], b[:3]):
        assert torch.equal(x, y)
    assert a[3] == b[3]


@pytest.mark.parametrize("form", ["graph", "pipelined2", "pipelined3", "pipelined3_defer", "pipelined3_fill"])
def test_overflowed_view_is_a_noop_for_the_optimizer(form, monkeypatch):
    """Capacities from the far views (headroom 1.0); the near view overflows: its replay leaves the
    language feature, both Adam moments and the device step count bit-unchanged, its gradient is zero
    (nothing was rasterized), the optimizer counts one skipped step, check() re-captures -- and the
    parameters then match the eager loop over the sequence WITHOUT that view.  _defer / _fill: the
    N > 1 structure (a GradBucket without a process group) with the deferred tail, whose skip word
    travels in the reduced partials (include/lsr.h LSR_BWD_DEFER_TAIL), or with LSR_PG_DEFER=0."""
    monkeypatch.setenv("LANGSPLAT_AMD_FUSED", "1")
    monkeypatch.setenv("LSR_PG_DEFER", "0" if form.endswith("_fill") else "1")
    P = 20000
    g = make_gaussians(P, seed=5, scale_range=(0.005, 0.04))
    views = _overflow_views()
    bad = 2
    kept = [v for i, v in enumerate(views) if i != bad]
    losses_e, se, _ = _eager_sequence(g, kept)
    m = _frozen_model(g)
    opt = _adam(m)
    fwd = _slot_forward(m)
    far_views = [v for i, v in enumerate(views) if i != bad]
    # capacities: the largest far view, no headroom
    R = E = 0
    for cam, gt, mask in far_views:
        mm = _frozen_model(g)
        with torch.no_grad():
            render(cam, mm, _Pipe, torch.zeros(3, device=DEV), _Opt, language_target=(gt, mask))
        r, e = _native.LAST_COUNTS[(P, 320, 240)]
        R, E = max(R, r), max(E, e)
    with torch.no_grad():
        render(views[bad][0], _frozen_model(g), _Pipe, torch.zeros(3, device=DEV), _Opt,
               language_target=views[bad][1:])
    assert _native.LAST_COUNTS[(P, 320, 240)][0] > 1.2 * R + 1024  # the near view needs more than the capacity
    snaps, losses = [], []
    if form == "graph":
        slot = ViewSlot(*views[0])

        def step():
            loss = fwd(slot)
            loss.backward()
            return loss
        gs = GraphedStep(step, [m._language_feature], optimizer=opt, view=slot, headroom=1.0)
        gs.capture(R, E)
        gs.headroom = 1.0
        for i, v in enumerate(views):
            snaps.append(_snap(m, opt))
            losses.append(gs.replay(view=v).clone())
            torch.cuda.synchronize()
            if i == bad:
                assert gs.overflow.view(torch.float32).item() == 1.0  # the bits of 1.0f (include/lsr.h)
                assert not m._language_feature.grad.any()  # nothing rasterized: a zero gradient
        snaps.append(_snap(m, opt))
        assert opt.skipped_steps() == 1
        assert not gs.check() and gs.captures == 2
    else:
        S = 2 if form == "pipelined2" else 3
        slots = [ViewSlot(*views[0]) for _ in range(S)]
        bucket = GradBucket([m._language_feature]) if "_" in form else None
        pg = PipelinedGraphStep(fwd, [m._language_feature], opt, slots=slots, headroom=1.0, bucket=bucket)
        pg.capture(R, E, views=views[:S - 1])
        assert pg.defer == form.endswith("_defer")
        L = S - 1
        for k in range(len(views)):
            snaps.append(_snap(m, opt))
            nxt = views[k + L] if k + L < len(views) else None
            losses.append(pg.replay(next_view=nxt).clone())
            pg.synchronize()
            torch.cuda.synchronize()
            if k == bad:
                assert pg.overflow[k % S].view(torch.float32).item() == 1.0
                assert not pg.last_grads()[0].any()
        snaps.append(_snap(m, opt))
        assert opt.skipped_steps() == 1
        assert not pg.check() and pg.captures == 2
    # the overflowed replay changed nothing; every other replay stepped
    _assert_bit_equal(snaps[bad], snaps[bad + 1])
    for i in range(len(views)):
        if i != bad:
            assert not torch.equal(snaps[i][0], snaps[i + 1][0]) and snaps[i + 1][3] == snaps[i][3] + 1
    opt.sync_steps()
    assert int(opt.state[m._language_feature]["step"].item()) == len(kept)
    got = [l for i, l in enumerate(losses) if i != bad]
    assert torch.equal(got[0], losses_e[0])
    torch.testing.assert_close(torch.stack(got), torch.stack(losses_e), rtol=1e-5, atol=0)
    assert_states_close(_state(m, opt), se, f"{form}, overflowed view left out")


# ---- Adam on the device: skip flag, learning-rate schedule, recapture --------------------------------

def test_captured_adam_skip_lr_schedule_and_recapture():
    """lsr_adam_multi with a device step block, captured: replays match torch.optim.Adam under a
    changing learning rate (sync_lr before each replay), a replay with the skip flag set changes
    nothing, eager steps interleave with replays, and a second prepare_capture (another capture of
    the same optimizer) leaves the first graph valid."""
    torch.manual_seed(0)
    n = 100003
    p0 = torch.randn(n, device=DEV)
    mine = torch.nn.Parameter(p0.clone())
    ref = torch.nn.Parameter(p0.clone())
    opt = Adam([{"params": [mine], "lr": 0.01, "name": "x"}], lr=0.0, eps=1e-15)
    topt = torch.optim.Adam([{"params": [ref], "lr": 0.01, "name": "x"}], lr=0.0, eps=1e-15, foreach=False)
    grads = [torch.randn(n, device=DEV) for _ in range(8)]
    gbuf = torch.zeros(n, device=DEV)
    skip = torch.zeros((), dtype=torch.int32, device=DEV)
    mine.grad = gbuf
    opt.prepare_capture()
    graph = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side), torch.cuda.graph(graph):
        opt.step(skip=skip)
    torch.cuda.current_stream().wait_stream(side)
    lrs = [0.01, 0.005, 0.002, 0.002, 0.001, 0.0005, 0.0005, 0.0001]

    def ref_step(k):
        for gr in topt.param_groups:
            gr["lr"] = lrs[k]
        ref.grad = grads[k].clone()
        topt.step()

    for k in range(3):
        opt.param_groups[0]["lr"] = lrs[k]
        gbuf.copy_(grads[k])
        opt.sync_lr()
        graph.replay()
        ref_step(k)
    torch.cuda.synchronize()
    torch.testing.assert_close(mine.detach(), ref.detach(), rtol=1e-6, atol=1e-7)
    # a skipped replay: bit-unchanged parameters, moments and count
    before = (mine.detach().clone(), opt.state[mine]["exp_avg"].clone(), opt.state[mine]["exp_avg_sq"].clone())
    skip.fill_(1)
    gbuf.copy_(grads[3])
    opt.sync_lr()
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(before[0], mine.detach()) and torch.equal(before[1], opt.state[mine]["exp_avg"])
    assert torch.equal(before[2], opt.state[mine]["exp_avg_sq"])
    assert opt.skipped_steps() == 1 and int(opt._step_dev[0].item()) == 3
    skip.fill_(0)
    # an eager step between replays continues the count (host and device)
    opt.param_groups[0]["lr"] = lrs[3]
    mine.grad = grads[3].clone()
    opt.step()
    ref_step(3)
    mine.grad = gbuf
    assert int(opt.state[mine]["step"].item()) == 4 and int(opt._step_dev[0].item()) == 4
    # another capture of the same optimizer: the device block is re-seeded in place
    opt.prepare_capture()
    for k in range(4, 8):
        opt.param_groups[0]["lr"] = lrs[k]
        gbuf.copy_(grads[k])
        opt.sync_lr()
        graph.replay()
        ref_step(k)
    torch.cuda.synchronize()
    opt.sync_steps()
    assert int(opt.state[mine]["step"].item()) == 8
    torch.testing.assert_close(mine.detach(), ref.detach(), rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(opt.state[mine]["exp_avg"], topt.state[ref]["exp_avg"], rtol=1e-5, atol=1e-8)
    torch.testing.assert_close(opt.state[mine]["exp_avg_sq"], topt.state[ref]["exp_avg_sq"], rtol=1e-5, atol=1e-10)


# ---- the fused language-step tail -----------------------------------------------------------------------

@pytest.mark.parametrize("form", ["graph", "pipelined2", "pipelined3"])
def test_fused_tail_matches_separate_launches(form, monkeypatch):
    """N = 1 captured steps apply Adam inside the backward's epilogue pass (include/lsr.h
    lsr_backward_args.update; the pipelined form also writes the updated feature into the next set's
    records, whose composite then skips its fill).  Against the same form with the separate epilogue,
    Adam and fill launches (LSR_FUSED_TAIL=0): the same losses, gradients, parameters and moments over
    five replays of a two-view sequence."""
    monkeypatch.setenv("LANGSPLAT_AMD_FUSED", "1")
    P, W, H = 60000, 640, 360
    g = make_gaussians(P, seed=9, scale_range=(0.004, 0.03))
    cams = make_cameras(8, W, H, device=DEV)
    views = []
    for v in (0, 3, 6, 1, 5):
        gt, mask = bench_target(H, W, v)
        views.append((cams[v], gt.to(DEV), mask.to(DEV)))
    runs = {}
    for fused in ("1", "0"):
        monkeypatch.setenv("LSR_FUSED_TAIL", fused)
        m = _frozen_model(g)
        opt = _adam(m, lr=0.01)
        fwd = _slot_forward(m)
        losses, grads = [], []
        if form == "graph":
            slot = ViewSlot(*views[0])

            def step():
                loss = fwd(slot)
                loss.backward()
                return loss
            gs = GraphedStep(step, [m._language_feature], optimizer=opt, view=slot).capture(1 << 22, 1 << 20)
            for v in views:
                losses.append(gs.replay(view=v).clone())
                grads.append(m._language_feature.grad.detach().clone())
            assert gs.check()
            gs.sync()
        else:
            S = int(form[-1])
            slots = [ViewSlot(*views[0]) for _ in range(S)]
            pg = PipelinedGraphStep(fwd, [m._language_feature], opt, slots=slots)
            pg.capture(1 << 22, 1 << 20, views=views[:S - 1])
            assert pg.fused == (fused == "1")
            for k in range(len(views)):
                nxt = views[k + S - 1] if k + S - 1 < len(views) else None
                losses.append(pg.replay(next_view=nxt).clone())
                grads.append(pg.last_grads()[0].detach().clone())  # read before set k % S is reused
            pg.synchronize()
            assert pg.check()
            pg.sync()
        torch.cuda.synchronize()
        assert int(opt.state[m._language_feature]["step"].item()) == len(views)
        runs[fused] = (torch.stack(losses), grads, _state(m, opt))
    (lf, gf, sf), (ls, gs_, ss) = runs["1"], runs["0"]
    assert torch.equal(lf[0], ls[0])  # the first step's loss: same bits (its gradient: float atomics)
    torch.testing.assert_close(lf, ls, rtol=1e-5, atol=0)
    for k, (a, b) in enumerate(zip(gf, gs_)):
        assert_grad_close(f"{form} step {k} language gradient", a.cpu().numpy(), b.cpu().numpy())
    assert_states_close(sf, ss, f"{form} fused vs separate tail")


# ---- a parameter changed by the caller between fused replays ----------------------------------------

@pytest.mark.parametrize("sets,rot", [(2, 1), (3, 1), (4, 2)])
def test_parameter_change_between_fused_replays(sets, rot, monkeypatch):
    """with the fused tail, step k writes the updated feature into the next set's
    records, whose composite (LSR_PHASE_COMPOSITE_FILLED) never re-reads the parameter.  The caller
    edits the language feature between replays and calls follow_caller(): the next replay refills
    those records from the parameter, so every loss and the final state equal the eager loop with the
    same edit at the same point (without the refill the next composite blends the stale feature)."""
    monkeypatch.setenv("LANGSPLAT_AMD_FUSED", "1")
    monkeypatch.setenv("LSR_FUSED_TAIL", "1")
    P, W, H = 60000, 640, 360
    g = make_gaussians(P, seed=9, scale_range=(0.004, 0.03))
    cams = make_cameras(8, W, H, device=DEV)
    views = []
    for v in (0, 3, 6, 1, 5, 2, 7, 4):
        gt, mask = bench_target(H, W, v)
        views.append((cams[v], gt.to(DEV), mask.to(DEV)))
    edit_after = 3  # a multiple of the rotation: edits land between rotation groups

    def edit(m):
        with torch.no_grad():
            m._language_feature.mul_(-0.5).add_(0.25)

    me = _frozen_model(g)
    oe = _adam(me, lr=0.01)
    losses_e = []
    for k, (cam, gt, mask) in enumerate(views):
        losses_e.append(_eager_step(me, oe, cam, gt, mask))
        if k + 1 == edit_after + (edit_after % rot):
            edit(me)
    se = _state(me, oe)
    m = _frozen_model(g)
    opt = _adam(m, lr=0.01)
    slots = [ViewSlot(*views[0]) for _ in range(sets)]
    pg = PipelinedGraphStep(_slot_forward(m), [m._language_feature], opt, slots=slots, rotation=rot)
    pg.capture(1 << 22, 1 << 20, views=views[:sets - 1])
    assert pg.fused
    losses = []
    for k in range(len(views)):
        nxt = views[k + sets - 1] if k + sets - 1 < len(views) else None
        losses.append(pg.replay(next_view=nxt).clone())
        if k + 1 == edit_after + (edit_after % rot):
            pg.synchronize()
            edit(m)
            pg.follow_caller()
    pg.synchronize()
    torch.cuda.synchronize()
    assert pg.check() and pg.captures == 1
    pg.sync()
    if rot == 1:
        torch.testing.assert_close(torch.stack(losses), torch.stack(losses_e), rtol=1e-5, atol=0)
    else:  # rotation: only the last R losses are still theirs
        torch.testing.assert_close(torch.stack(losses[-rot:]), torch.stack(losses_e[-rot:]), rtol=1e-5, atol=0)
    assert_states_close(_state(m, opt), se, f"edited between replays, {sets} sets, rotation {rot}")


# ---- the benched form over several steps at the reference's Adam eps ---------------------------------

def test_pipelined_graph_multi_step_at_reference_eps(monkeypatch):
    """bench.py's PipelinedGraphStep against the eager loop over K steps at C3 with
    the reference's Adam eps 1e-15 (scene/gaussian_model.py:229).  With eps 1e-15 Adam's first steps
    move an entry by ~lr sign(g) whatever |g| is, so an entry whose gradient is float-atomic noise
    takes a step of random sign in ANY two runs (eager against eager too).  The noise floor is
    measured here -- the largest difference between two backward passes of the same eager state,
    times 16 (measured on MI355X: 5.5e-12, floor 8.7e-11) -- and the parameters and moments are
    compared on the entries whose gradient exceeds it at every step (at least 100k entries; the
    language gradient is (1 / 3HW) per pixel times alpha T, so most entries of occluded or faint
    Gaussians sit near the floor)."""
    monkeypatch.setenv("LANGSPLAT_AMD_FUSED", "1")
    c = CONFIGS["C3"]
    P, W, H = c["P"], c["width"], c["height"]
    g = make_gaussians(P, seed=0)
    cam = make_cameras(1, W, H, device=DEV)[0]
    gt, mask = (t.to(DEV) for t in bench_target(H, W, 0))
    bg = torch.zeros(3, device=DEV)
    K = 4

    def adam(m):
        return Adam([{"params": [m._language_feature], "lr": LR, "name": "language_feature"}], lr=0.0, eps=1e-15)

    def fwd(m):
        return render(cam, m, _Pipe, bg, _Opt, language_target=(gt, mask))["language_l1"]
    # the float-atomic noise floor of this scene's gradient
    mn = _frozen_model(g)
    runs = []
    for _ in range(2):
        mn._language_feature.grad = None
        fwd(mn).backward()
        runs.append(mn._language_feature.grad.detach().clone())
    noise = float((runs[0] - runs[1]).abs().max())
    floor = 16.0 * max(noise, 1e-30)
    del mn, runs
    # eager steps, their gradients recorded
    me = _frozen_model(g)
    oe = adam(me)
    losses_e, above = [], None
    for _ in range(K):
        loss = fwd(me)
        loss.backward()
        gr = me._language_feature.grad.detach().abs() > floor
        above = gr if above is None else above & gr
        oe.step()
        oe.zero_grad(set_to_none=True)
        losses_e.append(loss.detach().clone())
        del loss
    se = _state(me, oe)
    # the benched form
    mg = _frozen_model(g)
    og = adam(mg)
    pg = PipelinedGraphStep(lambda: fwd(mg), [mg._language_feature], og).capture()
    assert pg.S == 3 and pg.fused
    losses = [pg.replay().clone() for _ in range(K)]
    pg.synchronize()
    torch.cuda.synchronize()
    assert pg.check()
    pg.sync()
    assert int(og.state[mg._language_feature]["step"].item()) == K
    sg = _state(mg, og)
    kept = above
    n_kept = int(kept.sum())
    print(f"noise floor {floor:.3e} (max two-run difference {noise:.3e}); entries above it at every step: "
          f"{n_kept} ({n_kept / kept.numel():.3f} of all)")
    assert n_kept >= 100_000, n_kept
    assert torch.equal(losses[0], losses_e[0])
    torch.testing.assert_close(torch.stack(losses), torch.stack(losses_e), rtol=1e-4, atol=0)
    for name, a, b, rtol, atol in (("param", sg[0], se[0], 1e-5, 1e-6), ("exp_avg", sg[1], se[1], 1e-4, 1e-9),
                                   ("exp_avg_sq", sg[2], se[2], 1e-4, 1e-12)):
        assert_close_mostly(f"eps 1e-15 {name}", a[kept], b[kept], rtol, atol)
