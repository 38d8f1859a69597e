"""Captured steps after a train.py-shaped eager loop (VERDICT r04 "next round" item 1).

LangSplat's train loop keeps the last iteration's render package and loss alive
(/root/reference/train.py:92-108: `render_pkg`, `loss` are reassigned, never deleted).  Those graphs
hold the language feature's AccumulateGrad node, bound to the stream the eager step ran on.  A capture
that reused the node made the captured backward wait on that non-capturing stream: torch warned
"AccumulateGrad node's stream does not match" and this HIP runtime segfaulted at capture end
(gpurun_out/r04_full1.log).  GraphedStep / PipelinedGraphStep.capture() now release
the parameters' cached nodes first (langsplat_amd/csrc/lsr_autograd.cpp).

Each test runs the eager loop, keeps its outputs, captures, replays, runs more eager iterations
(outputs kept again), then forces a library-side re-capture through check() with an over-capacity
view -- all with that warning turned into an error -- and compares the run with the eager loop over
the same views."""
import warnings

import pytest
import torch

from langsplat_amd import _native
from langsplat_amd.graph import GraphedStep, ViewSlot
from langsplat_amd.pipeline import PipelinedGraphStep
from langsplat_amd.render import render
from langsplat_amd.synthetic import make_gaussians
from tests.test_gpu_captured_forms import (_adam, _eager_sequence, _frozen_model, _overflow_views, _slot_forward,
                                           assert_states_close)
from tests.test_gpu_fused import _Opt, _Pipe

pytestmark = pytest.mark.gpu
DEV = "cuda"
MISMATCH = ".*AccumulateGrad node's stream does not match.*"


def _train_py_iteration(m, opt, view):
    """train.py:85-108 for one view: the render package and the loss are returned to the caller,
    who keeps them alive into the next iteration (as train.py's locals do)."""
    cam, gt, mask = view
    # train.py:138 leaves .grad None after every iteration; after replays the graph's own gradient
    # tensor sits there (graph.py: the graph owns it), which an eager backward would accumulate into
    opt.zero_grad(set_to_none=True)
    render_pkg = render(cam, m, _Pipe, torch.zeros(3, device=DEV), _Opt, language_target=(gt, mask))
    loss = render_pkg["language_l1"]
    loss.backward()
    opt.step()
    opt.zero_grad(set_to_none=True)
    return render_pkg, loss


def test_stale_node_is_bound_to_the_eager_stream():
    """The hazard itself: after an eager step whose outputs are kept, the parameter's cached node is
    bound to the caller's stream; release_stale_accumulators drops it, and a step on another stream
    then creates its own node there without the mismatch warning."""
    torch.autograd.graph.set_warn_on_accumulate_grad_stream_mismatch(True)
    A = _native.autograd_helper()
    g = make_gaussians(20000, seed=5, scale_range=(0.005, 0.04))
    m = _frozen_model(g)
    opt = _adam(m)
    views = _overflow_views()
    held = _train_py_iteration(m, opt, views[0])
    cur = torch.cuda.current_stream()
    assert A.accumulator_stream(m._language_feature) == (cur.device_index, cur.stream_id)
    from langsplat_amd.graph import release_stale_accumulators
    assert release_stale_accumulators([m._language_feature]) == 1
    side = torch.cuda.Stream()
    side.wait_stream(cur)
    with warnings.catch_warnings():
        warnings.filterwarnings("error", message=MISMATCH)
        with torch.cuda.stream(side):
            pkg = render(views[1][0], m, _Pipe, torch.zeros(3, device=DEV), _Opt, language_target=views[1][1:])
            assert A.accumulator_stream(m._language_feature) == (side.device_index, side.stream_id)
            pkg["language_l1"].backward()
    cur.wait_stream(side)
    torch.cuda.synchronize()
    assert held[1].grad_fn is not None  # the old graph is still alive


@pytest.mark.parametrize("form", ["graph", "pipelined3"])
def test_train_loop_then_capture_and_recapture(form, monkeypatch):
    monkeypatch.setenv("LANGSPLAT_AMD_FUSED", "1")
    torch.autograd.graph.set_warn_on_accumulate_grad_stream_mismatch(True)
    P = 20000
    g = make_gaussians(P, seed=5, scale_range=(0.005, 0.04))
    views = _overflow_views()  # view 2 is a near camera: several times the instances of the others
    bad = 2
    eager_views = views[:2]                         # the eager iterations before the capture
    replay_views = [views[3], views[4], views[bad], views[0], views[1]]
    mid_views = [views[3]]                          # eager iterations between replays and check()
    # the reference run: the eager loop over every view that gets trained, in the same order (the
    # over-capacity replay trains nothing)
    order = eager_views + [v for v in replay_views if v is not views[bad]]
    order = order[:4] + mid_views + order[4:]
    with warnings.catch_warnings():
        warnings.filterwarnings("error", message=MISMATCH)
        m = _frozen_model(g)
        opt = _adam(m)
        fwd = _slot_forward(m)
        # capacities from the far views (no headroom), so the near view overflows
        R = E = 0
        for cam, gt, mask in [v for i, v in enumerate(views) if i != bad]:
            with torch.no_grad():
                render(cam, _frozen_model(g), _Pipe, torch.zeros(3, device=DEV), _Opt, language_target=(gt, mask))
            r, e = _native.LAST_COUNTS[(P, 320, 240)]
            R, E = max(R, r), max(E, e)
        for v in eager_views:
            render_pkg, loss = _train_py_iteration(m, opt, v)  # kept alive, as in train.py
        assert render_pkg["language_l1"].grad_fn is not None and loss.grad_fn is not None
        if form == "graph":
            slot = ViewSlot(*replay_views[0])

            def step():
                loss = fwd(slot)
                loss.backward()
                return loss
            cap = GraphedStep(step, [m._language_feature], optimizer=opt, view=slot, headroom=1.0)
            cap.capture(R, E)
            assert cap.stale_released == 1
            losses = []
            for k, v in enumerate(replay_views[:2]):
                losses.append(cap.replay(view=v).clone())
            torch.cuda.synchronize()
            assert cap.check()
            cap.replay(view=replay_views[2])  # over capacity: skipped, flagged
            torch.cuda.synchronize()
            cap.sync()
            render_pkg, loss = _train_py_iteration(m, opt, mid_views[0])  # an eager step between, kept
            assert not cap.check() and cap.captures == 2  # the library-side re-capture
            for v in replay_views[3:]:
                losses.append(cap.replay(view=v).clone())
            torch.cuda.synchronize()
            assert cap.check()
            cap.sync()
        else:
            S = 3
            slots = [ViewSlot(*views[0]) for _ in range(S)]
            cap = PipelinedGraphStep(fwd, [m._language_feature], opt, slots=slots, headroom=1.0)
            cap.capture(R, E, views=replay_views[:S - 1])  # sets 0, 1: views 3, 4
            assert cap.stale_released == 1
            losses = []
            for k in range(3):  # trains views 3, 4; the third replay composites view 2: over capacity
                out = cap.replay(next_view=replay_views[k + S - 1]).clone()
                if k < 2:
                    losses.append(out)
            cap.synchronize()
            torch.cuda.synchronize()
            cap.sync()
            render_pkg, loss = _train_py_iteration(m, opt, mid_views[0])  # an eager step between, kept
            cap.follow_caller()  # the parameter changed on the caller's stream
            # the library-side re-capture, continuing with the views already loaded (0 and 1)
            assert not cap.check() and cap.captures == 2
            for _ in range(2):
                losses.append(cap.replay().clone())
            cap.synchronize()
            torch.cuda.synchronize()
            assert cap.check()
            cap.sync()
    # every iteration trained what the eager loop over `order` trains
    losses_e, se, _ = _eager_sequence(g, order)
    assert int(opt.state[m._language_feature]["step"].item()) == len(order)
    # the replays trained views 3, 4, then (after the eager step of view 3) 0, 1
    want = [losses_e[i] for i in (2, 3, 5, 6)]
    torch.testing.assert_close(torch.stack(losses), torch.stack(want), rtol=1e-5, atol=0)
    assert_states_close((m._language_feature.detach().clone(), opt.state[m._language_feature]["exp_avg"].clone(),
                         opt.state[m._language_feature]["exp_avg_sq"].clone()), se, f"{form} after re-capture")
