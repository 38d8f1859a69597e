"""The language step pipelined across views (langsplat_amd.pipeline.ViewPipeline): consecutive steps on
two alternating streams, the next view's geometry beside this view's backward and Adam, its
compositing behind the update (include/lsr.h lsr_forward_args.language_ready).  The pipeline only
reorders independent work: the first loss is bit-identical to the serial loop's, and later steps
agree to the rounding of the backward's float atomics (whose order varies between any two runs)."""
import pytest
import torch

from langsplat_amd.optim import Adam
from langsplat_amd.pipeline import ViewPipeline
from tests.test_gpu_graph import _language_setup

pytestmark = pytest.mark.gpu


def _run(mode, steps=6):
    m, step = _language_setup(P=5000)
    opt = Adam([{"params": [m._language_feature], "lr": 0.01, "name": "language_feature"}], lr=0.0, eps=1e-15)
    losses = []
    if mode == "serial":
        for _ in range(steps):
            losses.append(step().detach().clone())
            opt.step()
            opt.zero_grad(set_to_none=True)
    else:
        pipe = ViewPipeline(opt)
        for _ in range(steps):
            with pipe.step():
                losses.append(step().detach().clone())
                pipe.update()
        pipe.synchronize()
    torch.cuda.synchronize()
    st = opt.state[m._language_feature]
    return (m._language_feature.detach().clone(), st["exp_avg"].clone(), st["exp_avg_sq"].clone(),
            torch.stack(losses), int(st["step"].item()))


def test_view_pipeline_matches_serial_steps(monkeypatch):
    monkeypatch.setenv("LANGSPLAT_AMD_FUSED", "1")
    ps, ms, vs, ls, ns = _run("serial")
    po, mo, vo, lo, no = _run("pipelined")
    assert ns == no == 6
    assert torch.equal(ls[0], lo[0])
    torch.testing.assert_close(lo, ls, rtol=1e-5, atol=0)
    torch.testing.assert_close(po, ps, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(mo, ms, rtol=1e-4, atol=1e-9)
    torch.testing.assert_close(vo, vs, rtol=1e-4, atol=1e-12)


def test_view_pipeline_uses_two_streams(monkeypatch):
    """Steps alternate between the pipeline's two streams; update() outside a step is refused."""
    monkeypatch.setenv("LANGSPLAT_AMD_FUSED", "1")
    m, step = _language_setup(P=2000)
    opt = Adam([{"params": [m._language_feature], "lr": 0.01}], lr=0.0, eps=1e-15)
    pipe = ViewPipeline(opt)
    seen = []
    for _ in range(4):
        with pipe.step() as s:
            assert torch.cuda.current_stream() == s
            seen.append(s)
            step()
            pipe.update()
    assert seen[0] == seen[2] and seen[1] == seen[3] and seen[0] != seen[1]
    with pytest.raises(RuntimeError):
        pipe.update()
    pipe.synchronize()


def test_pipelined_graph_matches_serial_steps(monkeypatch):
    """PipelinedGraphStep: the forward split in its geometry and composite halves
    (lsr_forward_args.phase), the next view's geometry graph on its own stream beside this view's
    step graph.  After one eager step, K replays are K more serial steps: the same losses (the first
    bit for bit), parameters and Adam moments; the step count advanced on the device."""
    from langsplat_amd.pipeline import PipelinedGraphStep
    monkeypatch.setenv("LANGSPLAT_AMD_FUSED", "1")
    K = 5
    runs = {}
    for mode in ("serial", "graph"):
        m, step = _language_setup(P=5000)
        opt = Adam([{"params": [m._language_feature], "lr": 0.01, "name": "language_feature"}], lr=0.0, eps=1e-15)
        step()
        opt.step()
        opt.zero_grad(set_to_none=True)
        losses = []
        if mode == "serial":
            for _ in range(K):
                losses.append(step().detach().clone())
                opt.step()
                opt.zero_grad(set_to_none=True)
        else:
            g = PipelinedGraphStep(step.forward, [m._language_feature], opt).capture()
            for _ in range(K):
                losses.append(g.replay().clone())  # on the caller's stream: ordered after the replay
            g.synchronize()
            torch.cuda.synchronize()
            assert g.check() and g.captures == 1
            g.sync()
        st = opt.state[m._language_feature]
        runs[mode] = (m._language_feature.detach().clone(), st["exp_avg"].clone(), st["exp_avg_sq"].clone(),
                      torch.stack(losses), int(st["step"].item()))
    (ps, ms, vs, ls, ns), (pg, mg, vg, lg, ng) = runs["serial"], runs["graph"]
    assert ns == ng == K + 1
    assert torch.equal(ls[0], lg[0])
    torch.testing.assert_close(lg, ls, rtol=1e-5, atol=0)
    torch.testing.assert_close(pg, ps, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(mg, ms, rtol=1e-4, atol=1e-9)
    torch.testing.assert_close(vg, vs, rtol=1e-4, atol=1e-12)


def test_forward_phases_match_one_call(monkeypatch):
    """lsr_forward in two calls (GEOMETRY, then COMPOSITE into the same static buffers) produces the
    one-call capacity-mode forward's image, language image, radii and loss bit for bit, and the
    backward over it the same gradients; a phase outside capacity mode is refused."""
    from langsplat_amd import _native
    monkeypatch.setenv("LANGSPLAT_AMD_FUSED", "1")
    m, step = _language_setup(P=5000)
    outs = []
    for split in (False, True):
        sb = _native.static_buffers()
        ov = torch.zeros((), dtype=torch.int32, device="cuda")
        m._language_feature.grad = None
        with _native.capacity(1 << 20, 1 << 20, ov), sb:
            if split:
                with _native.forward_phase(_native.forward_phase.GEOMETRY):
                    step.forward()
                with _native.forward_phase(_native.forward_phase.COMPOSITE):
                    loss = step.forward()
            else:
                loss = step.forward()
            loss.backward()
        torch.cuda.synchronize()
        assert int(ov.item()) == 0
        outs.append((loss.detach().clone(), sb.tensors[("out", "color")].clone(),
                     sb.tensors[("out", "language")].clone(), sb.tensors[("out", "radii")].clone(),
                     m._language_feature.grad.detach().clone()))
    (l0, c0, f0, r0, g0), (l1, c1, f1, r1, g1) = outs
    assert torch.equal(l0, l1) and torch.equal(c0, c1) and torch.equal(f0, f1) and torch.equal(r0, r1)
    torch.testing.assert_close(g1, g0, rtol=1e-5, atol=1e-9)
    with pytest.raises(RuntimeError, match="phase"):
        with _native.forward_phase(_native.forward_phase.GEOMETRY):
            step.forward()
