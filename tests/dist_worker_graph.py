"""One rank of the N = 2 RGB step captured by GraphedStep(bucket=) across a reset_opacity, for
tests/test_gpu_dist_step.py (not a test).  ADVICE r05: a re-capture after the parameters were
replaced must reduce the NEW tensors' gradients (bucket_factory), or refuse (no factory).

    LSR_DIST_BACKEND=gloo python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
        tests/dist_worker_graph.py OUT_DIR

Each rank renders camera `rank` of a small scene and runs SCHEDULE twice: eagerly (render + L1,
backward, GradBucket all-reduce, [reset_opacity], Adam; a new bucket after the reset) and with
GraphedStep(bucket=, bucket_factory=) replays (the reset iteration eager, as the reference's
iteration does it between backward and step).  Writes OUT_DIR/graph<r>.pt: both forms' parameters
and step counts, the number of captures, and whether a GraphedStep without a factory refused the
stale bucket."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from langsplat_amd.densify import Densifier  # noqa: E402
from langsplat_amd.distributed import GradBucket, init_from_env  # noqa: E402
from langsplat_amd.graph import GraphedStep  # noqa: E402
from langsplat_amd.synthetic import make_cameras, make_gaussians  # noqa: E402
from tests.test_gpu_train_loop import ATTRS, _loss, _rgb  # noqa: E402

SCHEDULE = [False, False, True, False, False]  # reset_opacity inside the third iteration


def params_of(m):
    return [getattr(m, a) for a in ATTRS.values()]


def run(form, g, cam, gt, factory=True):
    m, opt = _rgb(g)
    m.active_sh_degree = 1

    def step():
        loss = _loss(m, cam, gt)
        loss.backward()
        return loss

    bucket = GradBucket(params_of(m))
    gs = None
    for reset in SCHEDULE:
        if form == "eager" or reset:
            if gs is not None:
                gs.sync()
                bucket = gs.bucket
            opt.zero_grad(set_to_none=True)
            step()
            bucket.all_reduce(average=True)
            if reset:
                Densifier(m, opt).reset_opacity()
            opt.step()
            opt.zero_grad(set_to_none=True)
            if form == "eager" and not bucket.matches(params_of(m)):
                bucket = GradBucket(params_of(m))
        else:
            if gs is None:
                gs = GraphedStep(step, params_of(m), optimizer=opt, model=m, bucket=bucket,
                                 bucket_factory=(lambda ps: GradBucket(ps)) if factory else None)
            gs.replay()
    torch.cuda.synchronize()
    caps = 0
    if gs is not None:
        assert gs.check()
        gs.sync()
        caps = gs.captures
    return ({n: getattr(m, a).detach().cpu() for n, a in ATTRS.items()},
            {n: int(opt.state[getattr(m, a)]["step"].item()) for n, a in ATTRS.items()}, caps)


def main():
    out_dir = sys.argv[1]
    rank, world = init_from_env()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    P, W, H = 20000, 256, 192
    g = make_gaussians(P, seed=21, scale_range=(0.005, 0.05))
    cam = make_cameras(8, W, H, device=dev)[rank]
    gt = torch.rand((3, H, W), generator=torch.Generator().manual_seed(3 + rank)).to(dev)
    out = {}
    for form in ("eager", "graph"):
        out[form] = run(form, g, cam, gt)
    try:  # the same replays without a factory: the re-capture after the reset must refuse
        run("graph", g, cam, gt, factory=False)
        out["refused"] = False
    except RuntimeError as e:
        out["refused"] = "bucket_factory" in str(e)
    torch.save(out, os.path.join(out_dir, f"graph{rank}.pt"))
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
