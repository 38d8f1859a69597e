"""One rank of the N = 2 language step on one GPU, for tests/test_gpu_dist_step.py (not a test).

    LSR_DIST_BACKEND=gloo python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
        tests/dist_worker.py OUT_DIR

Each rank trains BASELINE.json configs[3] (C4: 1M Gaussians, 1920x1080) on camera `rank` of 8 with
bench.py's synthetic language target of that view, in two step forms bench.py times at N > 1:
  eager            render + fused loss, backward, GradBucket.all_reduce (average), Adam;
  pipelined_graph  langsplat_amd.pipeline.PipelinedGraphStep(..., bucket=): the backward and Adam
                   graphs of the view's buffer set with the all-reduce launched between them (the
                   deferred tail: the collective over the backward's language partials);
  pipelined_graph_fill  the same with LSR_PG_DEFER=0 (the collective over .grad);
  multi_step       four steps of the eager loop and of the deferred-tail pipelined graph at Adam eps
                   1e-15, with the entries above the float-atomic noise floor.
After one step each rank writes OUT_DIR/rank<r>.pt with the averaged language gradient, the loss and
the updated parameter of both forms."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from langsplat_amd.distributed import GradBucket, init_from_env  # noqa: E402
from langsplat_amd.optim import Adam  # noqa: E402
from langsplat_amd.pipeline import PipelinedGraphStep  # noqa: E402
from langsplat_amd.render import render  # noqa: E402
from langsplat_amd.synthetic import CONFIGS, make_cameras, make_gaussians  # noqa: E402
from tests.test_gpu_fused import _Model, _Opt, _Pipe  # noqa: E402
from tests.test_gpu_timed_step import bench_target  # noqa: E402

LR = 0.0025


def frozen_model(g, dev):
    m = _Model(g, dev)
    for n in ("xyz", "features_dc", "features_rest", "scaling", "rotation", "opacity"):
        getattr(m, "_" + n).requires_grad_(False)
    return m


def main():
    out_dir = sys.argv[1]
    rank, world = init_from_env()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    c = CONFIGS["C4"]
    P, W, H = c["P"], c["width"], c["height"]
    g = make_gaussians(P, seed=0)
    cam = make_cameras(c["views"], W, H, device=dev)[rank]
    gt, mask = (t.to(dev) for t in bench_target(H, W, rank))
    bg = torch.zeros(3, device=dev)
    out = {}
    # eager: render + loss + backward, all-reduce, Adam
    m = frozen_model(g, dev)
    opt = Adam([{"params": [m._language_feature], "lr": LR, "name": "language_feature"}], lr=0.0, eps=1e-8)
    bucket = GradBucket([m._language_feature])
    loss = render(cam, m, _Pipe, bg, _Opt, language_target=(gt, mask))["language_l1"]
    loss.backward()
    bucket.all_reduce(average=True)
    grad = m._language_feature.grad.detach().clone()
    opt.step()
    torch.cuda.synchronize()
    out["eager"] = dict(grad=grad.cpu(), loss=loss.detach().cpu(), param=m._language_feature.detach().cpu())
    del m, opt, bucket, loss
    # the pipelined graph form with the all-reduce between its backward and Adam graphs: the deferred
    # tail (the collective over the backward's language partials, then one pass: gradients, Adam,
    # fill; include/lsr.h LSR_BWD_DEFER_TAIL) and, LSR_PG_DEFER=0, the epilogue before the collective
    for form, defer in (("pipelined_graph", "1"), ("pipelined_graph_fill", "0")):
        os.environ["LSR_PG_DEFER"] = defer
        m = frozen_model(g, dev)
        opt = Adam([{"params": [m._language_feature], "lr": LR, "name": "language_feature"}], lr=0.0, eps=1e-8)
        bucket = GradBucket([m._language_feature])
        pg = PipelinedGraphStep(lambda: render(cam, m, _Pipe, bg, _Opt, language_target=(gt, mask))["language_l1"],
                                [m._language_feature], opt, bucket=bucket).capture()
        assert pg.defer == (defer == "1")
        loss = pg.replay().clone()
        pg.synchronize()
        torch.cuda.synchronize()
        assert pg.check()
        pg.sync()
        out[form] = dict(grad=pg.last_grads()[0].detach().cpu(), loss=loss.cpu(),
                         param=m._language_feature.detach().cpu(),
                         step=int(opt.state[m._language_feature]["step"].item()))
        del pg, m, opt, bucket
    # K steps at the reference's Adam eps 1e-15 (scene/gaussian_model.py:229): the eager loop and the
    # deferred-tail pipelined graph, with the entries whose averaged gradient stays above the
    # float-atomic noise floor at every step (tests/test_gpu_captured_forms.py
    # test_pipelined_graph_multi_step_at_reference_eps explains the floor)
    os.environ["LSR_PG_DEFER"] = "1"
    K = 4

    def adam15(m):
        return Adam([{"params": [m._language_feature], "lr": LR, "name": "language_feature"}], lr=0.0, eps=1e-15)

    def fwd(m):
        return render(cam, m, _Pipe, bg, _Opt, language_target=(gt, mask))["language_l1"]
    mn = frozen_model(g, dev)
    runs = []
    for _ in range(2):
        mn._language_feature.grad = None
        fwd(mn).backward()
        runs.append(mn._language_feature.grad.detach().clone())
    floor = 16.0 * max(float((runs[0] - runs[1]).abs().max()), 1e-30)
    del mn, runs
    me = frozen_model(g, dev)
    oe = adam15(me)
    be = GradBucket([me._language_feature])
    above = None
    for _ in range(K):
        fwd(me).backward()
        be.all_reduce(average=True)
        gr = me._language_feature.grad.detach().abs() > floor
        above = gr if above is None else above & gr
        oe.step()
        oe.zero_grad(set_to_none=True)
    st = oe.state[me._language_feature]
    ref = (me._language_feature.detach().cpu(), st["exp_avg"].cpu(), st["exp_avg_sq"].cpu())
    mg = frozen_model(g, dev)
    og = adam15(mg)
    pg = PipelinedGraphStep(lambda: fwd(mg), [mg._language_feature], og, bucket=GradBucket([mg._language_feature])).capture()
    assert pg.defer
    for _ in range(K):
        pg.replay()
    pg.synchronize()
    torch.cuda.synchronize()
    assert pg.check()
    pg.sync()
    st = og.state[mg._language_feature]
    out["multi_step"] = dict(eager=ref, graph=(mg._language_feature.detach().cpu(), st["exp_avg"].cpu(),
                                               st["exp_avg_sq"].cpu()),
                             above=above.cpu(), step=int(st["step"].item()), floor=floor)
    torch.save(out, os.path.join(out_dir, f"rank{rank}.pt"))
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
