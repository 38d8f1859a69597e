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
    """PipelinedGraphStep: after one eager step, the capture's prologue forward composites view 1 and
    replay r runs view r's backward and Adam, then view r+1's forward -- so the losses it leaves in the
    two buffer sets and the parameters after K replays are those of K more serial steps."""
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
            losses.append(step().detach().clone())  # view K + 1's loss (the last replay's forward)
            m._language_feature.grad = None
        else:
            g = PipelinedGraphStep(step.forward, [m._language_feature], opt).capture()
            torch.cuda.synchronize()
            losses.append(g.static_loss[0].clone())  # the prologue's view
            for _ in range(K):
                loss = g.replay()
                g.synchronize()  # the loss is written on the pipeline's forward stream
                losses.append(loss.clone())
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
