"""View-sharded data parallelism on CPU (gloo, world_size 2 and 3): the all-reduced gradient
bucket equals the sum of the per-view single-process gradients (SURVEY.md §8e parity)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from langsplat_amd.distributed import GradBucket


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _view_grads(view, n_views):
    """Oracle gradients of one view w.r.t. (language feature, opacity) of a shared scene."""
    from oracle import oracle
    from tests.scenes import grad_seed, scene
    st, inp = scene(P=150, W=40, H=32, seed=0, view=view, n_views=n_views, scale_range=(0.05, 0.25))
    run = oracle.forward(st, **inp)
    gc, gl = grad_seed(32, 40, seed=10 + view)
    g = run.backward(gc, gl)
    return torch.tensor(g["language_feature_precomp"]), torch.tensor(g["opacities"])


def _worker(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lang = torch.nn.Parameter(torch.zeros((150, 3)))
        opac = torch.nn.Parameter(torch.zeros((150, 1)))
        frozen = torch.nn.Parameter(torch.zeros((150, 3)), requires_grad=False)
        bucket = GradBucket([lang, frozen, opac])
        assert bucket.nbytes == 150 * 4 * 4
        gl, go = _view_grads(rank, world)
        # autograd-style in-place accumulation into the bucket-backed .grad tensors
        lang.grad.add_(gl)
        opac.grad.add_(go)
        bucket.all_reduce(average=False)
        np.save(os.path.join(out_dir, f"lang_{rank}.npy"), lang.grad.numpy())
        np.save(os.path.join(out_dir, f"opac_{rank}.npy"), opac.grad.numpy())
        bucket.zero()
        lang.grad.add_(gl)
        opac.grad.add_(go)
        bucket.all_reduce(average=True)
        np.save(os.path.join(out_dir, f"lang_avg_{rank}.npy"), lang.grad.numpy())
        # a detached .grad is reported instead of silently reducing a stale buffer
        lang.grad = None
        try:
            bucket.all_reduce()
            raise AssertionError("expected RuntimeError")
        except RuntimeError:
            pass
        # one trainable parameter (the language-feature step): direct mode reduces the .grad
        # autograd left (zero_grad(set_to_none=True): a fresh tensor each step) in place
        lang1 = torch.nn.Parameter(torch.zeros((150, 3)))
        direct = GradBucket([lang1, frozen])
        assert direct.direct and direct.flat is None and direct.nbytes == 150 * 3 * 4
        lang1.grad = gl.clone()
        direct.all_reduce(average=False)
        np.save(os.path.join(out_dir, f"direct_{rank}.npy"), lang1.grad.numpy())
        lang1.grad = None  # set_to_none: nothing to reduce is an error, not a silent no-op
        try:
            direct.all_reduce()
            raise AssertionError("expected RuntimeError")
        except RuntimeError:
            pass
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_allreduced_bucket_equals_sum_of_view_gradients(tmp_path, world):
    port = _free_port()
    mp.spawn(_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    ref_l = sum(_view_grads(v, world)[0] for v in range(world)).numpy()
    ref_o = sum(_view_grads(v, world)[1] for v in range(world)).numpy()
    for r in range(world):
        np.testing.assert_allclose(np.load(tmp_path / f"lang_{r}.npy"), ref_l, rtol=1e-5, atol=1e-8)
        np.testing.assert_allclose(np.load(tmp_path / f"opac_{r}.npy"), ref_o, rtol=1e-5, atol=1e-8)
        np.testing.assert_allclose(np.load(tmp_path / f"lang_avg_{r}.npy"), ref_l / world, rtol=1e-5, atol=1e-8)
        np.testing.assert_allclose(np.load(tmp_path / f"direct_{r}.npy"), ref_l, rtol=1e-5, atol=1e-8)
    # the ranks agree bit for bit (one collective, same result everywhere; float sums in ring order)
    for r in range(1, world):
        assert np.array_equal(np.load(tmp_path / f"lang_{r}.npy"), np.load(tmp_path / "lang_0.npy"))


def test_bucket_requires_trainable_fp32():
    with pytest.raises(ValueError):
        GradBucket([torch.nn.Parameter(torch.zeros(3), requires_grad=False)])
    with pytest.raises(TypeError):
        GradBucket([torch.nn.Parameter(torch.zeros(3, dtype=torch.float64))])
