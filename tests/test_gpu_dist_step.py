"""bench.py's N = 2 language step as two gloo ranks sharing cuda:0.

tests/dist_worker.py runs, on each rank, camera `rank` of C4 (BASELINE.json configs[3]) through the
eager step (render + fused loss, backward, GradBucket all-reduce, Adam) and through the pipelined
graph form with the all-reduce launched between its backward and Adam graphs.  The averaged
language gradient must equal the mean of the two views' oracle gradients (the per-view oracle step of
tests/test_gpu_timed_step.py), be identical on both ranks, and leave both ranks with identical
parameters.  gloo reduces on the host: this checks the N > 1 data flow, not RCCL's speed (the RCCL
path itself runs in tests/test_gpu_rccl.py)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from langsplat_amd.synthetic import CONFIGS, make_cameras, make_gaussians
from tests.test_gpu_parity import assert_grad_close
from tests.test_gpu_timed_step import bench_target, oracle_language_step

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_rank_language_step_averages_the_views_gradients(tmp_path):
    env = dict(os.environ, LSR_DIST_BACKEND="gloo", LANGSPLAT_AMD_FUSED="1", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "dist_worker.py"), str(tmp_path)]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    outs = [torch.load(tmp_path / f"rank{k}.pt", weights_only=True) for k in (0, 1)]
    c = CONFIGS["C4"]
    P, W, H = c["P"], c["width"], c["height"]
    g = make_gaussians(P, seed=0)
    cams = make_cameras(c["views"], W, H)
    refs = []
    for v in (0, 1):
        gt, mask = bench_target(H, W, v)
        run, loss_ref, d_lang, _ = oracle_language_step(g, cams[v], gt, mask)
        refs.append((loss_ref, d_lang))
        del run
    mean = 0.5 * (refs[0][1].astype(np.float64) + refs[1][1].astype(np.float64))
    for form in ("eager", "pipelined_graph", "pipelined_graph_fill"):
        for k in (0, 1):
            o = outs[k][form]
            # each rank's own loss is its view's
            assert abs(float(o["loss"]) - refs[k][0]) <= 2e-6 * refs[k][0], (form, k)
            assert_grad_close(f"{form} rank {k} averaged language gradient", o["grad"].numpy(), mean)
        assert torch.equal(outs[0][form]["grad"], outs[1][form]["grad"]), form
        assert torch.equal(outs[0][form]["param"], outs[1][form]["param"]), form
    assert outs[0]["pipelined_graph"]["step"] == outs[0]["pipelined_graph_fill"]["step"] == 1
    # the forms take the same Adam step from the same averaged gradient (to its rounding: Adam's
    # first step is lr * g / |g|, so an entry whose gradient cancels to ~0 may differ in sign; the
    # deferred tail averages the partials before the activation's chain rule, the others after it)
    for form in ("pipelined_graph", "pipelined_graph_fill"):
        a, b = outs[0][form]["param"].double(), outs[0]["eager"]["param"].double()
        off = int(((a - b).abs() > 1e-6 + 1e-5 * b.abs()).sum())
        assert off <= 1e-5 * a.numel(), (form, off)
    # four steps at the reference's eps 1e-15: the deferred-tail graph against the eager loop on the
    # entries above the noise floor (at least 100k), and identical ranks
    from tests.test_gpu_captured_forms import assert_close_mostly
    for k in (0, 1):
        ms = outs[k]["multi_step"]
        assert ms["step"] == 4
        kept = ms["above"]
        assert int(kept.sum()) >= 100_000, int(kept.sum())
        for name, a, b, rtol, atol in zip(("param", "exp_avg", "exp_avg_sq"), ms["graph"], ms["eager"],
                                          (1e-5, 1e-4, 1e-4), (1e-6, 1e-9, 1e-12)):
            assert_close_mostly(f"rank {k} {name}", a[kept], b[kept], rtol=rtol, atol=atol)
    for i in range(3):
        assert torch.equal(outs[0]["multi_step"]["graph"][i], outs[1]["multi_step"]["graph"][i])


def test_two_rank_graphed_rgb_step_rebuilds_its_bucket_after_reset_opacity(tmp_path):
    """GraphedStep(bucket=) re-captured after reset_opacity replaced the opacity tensor
    reduces the new tensor's gradient through a bucket rebuilt by bucket_factory (both ranks end
    identical and equal to the eager loop with its own rebuilt bucket), and refuses without one."""
    env = dict(os.environ, LSR_DIST_BACKEND="gloo", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "dist_worker_graph.py"), str(tmp_path)]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    outs = [torch.load(tmp_path / f"graph{k}.pt", weights_only=True) for k in (0, 1)]
    from tests.test_gpu_captured_forms import assert_close_mostly
    for o in outs:
        assert o["refused"]
        (pe, se, _), (pg, sg, caps) = o["eager"], o["graph"]
        assert se == sg and se["opacity"] == se["xyz"] - 1  # the reset iteration left opacity out
        assert caps == 2  # the first capture and the one after the reset
        for n in pe:
            assert_close_mostly(n, pg[n], pe[n], rtol=1e-5, atol=1e-6, outliers=1e-4)
    for form in ("eager", "graph"):
        for n, v in outs[0][form][0].items():
            assert torch.equal(v, outs[1][form][0][n]), (form, n)  # the ranks stay identical
