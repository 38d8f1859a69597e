"""View-sharded data parallelism on CPU (gloo, world_size 2, 3 and 8 -- north_star's 8-view
partitioning): the all-reduced gradient bucket equals the sum of the per-view
single-process gradients (SURVEY.md §8e parity)."""
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
        # zero_grad(set_to_none=True) detaches the .grad tensors from the bucket: the next all_reduce
        # re-attaches them (a fresh .grad is copied into its slice, a missing one reduces as zeros), so
        # no rank raises while the others wait inside the collective
        bucket.zero()
        lang.grad = None
        opac.grad = go.clone()  # a fresh tensor, as autograd leaves after set_to_none
        bucket.all_reduce(average=False)
        assert bucket.attached() and not lang.grad.any()
        np.save(os.path.join(out_dir, f"reattach_{rank}.npy"), opac.grad.numpy())
        # one trainable parameter (the language-feature step): direct mode reduces the .grad
        # autograd left (zero_grad(set_to_none=True): a fresh tensor each step) in place
        lang1 = torch.nn.Parameter(torch.zeros((150, 3)))
        direct = GradBucket([lang1, frozen])
        assert direct.direct and direct.flat is None and direct.nbytes == 150 * 3 * 4
        lang1.grad = gl.clone()
        direct.all_reduce(average=False)
        np.save(os.path.join(out_dir, f"direct_{rank}.npy"), lang1.grad.numpy())
        # a rank whose parameter got no gradient this step joins with zeros (rank 0 here)
        lang1.grad = None if rank == 0 else gl.clone()
        direct.all_reduce(average=False)
        np.save(os.path.join(out_dir, f"direct_none_{rank}.npy"), lang1.grad.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
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
        np.testing.assert_allclose(np.load(tmp_path / f"reattach_{r}.npy"), ref_o, rtol=1e-5, atol=1e-8)
        ref_none = sum(_view_grads(v, world)[0] for v in range(1, world)).numpy()
        np.testing.assert_allclose(np.load(tmp_path / f"direct_none_{r}.npy"), ref_none, rtol=1e-5, atol=1e-8)
    # the ranks agree bit for bit (one collective, same result everywhere; float sums in ring order)
    for r in range(1, world):
        assert np.array_equal(np.load(tmp_path / f"lang_{r}.npy"), np.load(tmp_path / "lang_0.npy"))


def test_bucket_requires_trainable_fp32():
    with pytest.raises(ValueError):
        GradBucket([torch.nn.Parameter(torch.zeros(3), requires_grad=False)])
    with pytest.raises(TypeError):
        GradBucket([torch.nn.Parameter(torch.zeros(3, dtype=torch.float64))])


def _view_stats(view, n_views):
    """One view's radii and dL/dmeans2D (oracle) of the shared densification scene."""
    from oracle import oracle
    from tests.scenes import grad_seed, scene
    st, inp = scene(P=200, W=48, H=40, seed=1, view=view, n_views=n_views, scale_range=(0.05, 0.25))
    run = oracle.forward(st, **inp)
    gc, gl = grad_seed(40, 48, seed=20 + view)
    g = run.backward(gc, gl)
    return torch.tensor(run.radii), torch.tensor(g["means2D"])


def _densify_worker(rank, world, port, out_dir, average):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        P = 200
        xyz = torch.nn.Parameter(torch.zeros((P, 3)))
        opac = torch.nn.Parameter(torch.zeros((P, 1)))
        bucket = GradBucket([xyz, opac], densify_points=P)
        accum, denom = torch.full((P, 1), 0.25), torch.full((P, 1), 2.0)   # earlier iterations' sums
        max_radii = torch.full((P,), 3.0)
        for step in range(2):  # the statistics of two steps accumulate; the bucket is zeroed between
            bucket.zero()
            radii, dm2 = _view_stats(rank + world * step, 2 * world)
            xyz.grad.add_(dm2)
            bucket.stage_densification(radii, dm2, max_radii)
            bucket.all_reduce(average=average)
            bucket.apply_densification(accum, denom)
        np.save(os.path.join(out_dir, f"accum_{rank}.npy"), accum.numpy())
        np.save(os.path.join(out_dir, f"denom_{rank}.npy"), denom.numpy())
        np.save(os.path.join(out_dir, f"maxr_{rank}.npy"), max_radii.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,average", [(2, True), (3, True), (3, False), (8, True)])
def test_densification_statistics_sum_over_views(tmp_path, world, average):
    """RGB-mode densification statistics (train.py:125-126, scene/gaussian_model.py:480-482) over
    view-sharded ranks equal the reference's accumulation over the same views done one after
    another: SUM of ||dL/dmeans2D[:, :2]|| and of the visibility counts, MAX of the radii."""
    P = 200
    port = _free_port()
    mp.spawn(_densify_worker, args=(world, port, str(tmp_path), average), nprocs=world, join=True)
    accum, denom = torch.full((P, 1), 0.25, dtype=torch.float64), torch.full((P, 1), 2.0, dtype=torch.float64)
    max_radii = torch.full((P,), 3.0, dtype=torch.float64)
    for v in range(2 * world):  # the reference: one view per iteration
        radii, dm2 = _view_stats(v, 2 * world)
        vis = radii > 0
        max_radii[vis] = torch.max(max_radii[vis], radii[vis].double())
        accum[vis] += torch.norm(dm2[vis, :2].double(), dim=-1, keepdim=True)
        denom[vis] += 1
    for r in range(world):
        np.testing.assert_allclose(np.load(tmp_path / f"accum_{r}.npy"), accum.numpy(), rtol=1e-5, atol=1e-9)
        np.testing.assert_array_equal(np.load(tmp_path / f"denom_{r}.npy"), denom.numpy().astype(np.float32))
        np.testing.assert_array_equal(np.load(tmp_path / f"maxr_{r}.npy"), max_radii.numpy().astype(np.float32))
    assert denom.max() > 2.0 + world  # the views overlap: some Gaussians counted by several ranks


def _flag_worker(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lang = torch.nn.Parameter(torch.zeros((150, 3)))
        opac = torch.nn.Parameter(torch.zeros((150, 1)))
        out = {}
        for mode, params in (("direct", [lang]), ("flat", [lang, opac])):
            bucket = GradBucket(params)
            assert bucket.direct == (mode == "direct")
            for step, over in enumerate((None, world - 1)):  # no rank overflows, then only the last one
                bucket.zero()
                lang.grad = torch.full((150, 3), float(rank + 1)) if bucket.direct else lang.grad.add_(rank + 1)
                # the rasterizer's overflow flag: 0, or the bits of 1.0f (include/lsr.h)
                flag = torch.tensor(0x3F800000 if rank == over else 0, dtype=torch.int32)
                bucket.all_reduce(average=True, flag=flag)
                out[f"{mode}{step}_grad"] = lang.grad.clone()
                out[f"{mode}{step}_flag"] = int(flag.item())
        # the deferred language tail (include/lsr.h LSR_BWD_DEFER_TAIL): ONE all-reduce over the backward's
        # 3 P language partials followed by the skip word, which carries the overflow flag itself
        bucket = GradBucket([lang])
        from langsplat_amd import rccl
        assert not rccl.direct_enabled()  # gloo: torch.distributed's all-reduce (the direct one is RCCL's)
        for step, over in enumerate((None, world - 1)):
            part = torch.full((3 * 150 + 1,), float(rank + 1))
            part[-1:].view(torch.int32)[0] = 0x3F800000 if rank == over else 0
            bucket.all_reduce_partials(part, average=True)
            out[f"partials{step}_grad"] = part[:-1].clone()
            out[f"partials{step}_flag"] = int(part[-1:].view(torch.int32).item())
        torch.save(out, os.path.join(out_dir, f"flag_{rank}.pt"))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_overflow_flag_rides_the_gradient_collective(tmp_path, world):
    """a view over capacity on ONE rank sets the flag on EVERY rank (the flag is
    all-reduced in the same collective as the gradients), so every rank skips the optimizer step and
    the ranks stay identical; the gradients are averaged as without the flag (direct and flat).  Also
    the deferred tail's collective (round 6): the language partials with the skip word after them."""
    port = _free_port()
    mp.spawn(_flag_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    outs = [torch.load(tmp_path / f"flag_{r}.pt", weights_only=True) for r in range(world)]
    mean = sum(range(1, world + 1)) / world
    for o in outs:
        for mode in ("direct", "flat"):
            assert o[f"{mode}0_flag"] == 0
            assert o[f"{mode}1_flag"] != 0  # non-zero as an int: Adam's skip test
            for step in (0, 1):
                torch.testing.assert_close(o[f"{mode}{step}_grad"], torch.full((150, 3), mean))
        assert o["partials0_flag"] == 0 and o["partials1_flag"] != 0
        for step in (0, 1):
            torch.testing.assert_close(o[f"partials{step}_grad"], torch.full((450,), mean))
    for r in range(1, world):
        for k, v in outs[r].items():
            assert (torch.equal(v, outs[0][k]) if torch.is_tensor(v) else v == outs[0][k]), k


def test_bucket_matches_and_is_rebuilt_after_parameter_replacement():
    """a capture over replaced parameters (reset_opacity, densify_and_prune) must not keep
    a bucket built over the old tensors: resolve_bucket keeps a matching bucket, rebuilds with the
    factory, and raises without one."""
    from langsplat_amd.graph import resolve_bucket
    xyz = torch.nn.Parameter(torch.zeros((10, 3)))
    opac = torch.nn.Parameter(torch.zeros((10, 1)))
    b = GradBucket([xyz, opac], densify_points=10)
    assert b.matches([xyz, opac]) and resolve_bucket(b, None, [xyz, opac]) is b
    new_opac = torch.nn.Parameter(torch.zeros((10, 1)))  # reset_opacity: same shape, a new tensor
    assert not b.matches([xyz, new_opac])
    with pytest.raises(RuntimeError, match="bucket_factory"):
        resolve_bucket(b, None, [xyz, new_opac])
    nb = resolve_bucket(b, lambda ps: GradBucket(ps, densify_points=ps[0].shape[0]), [xyz, new_opac])
    assert nb is not b and nb.matches([xyz, new_opac]) and new_opac.grad.data_ptr() == nb.views[1].data_ptr()
    grown = [torch.nn.Parameter(torch.zeros((12, 3))), torch.nn.Parameter(torch.zeros((12, 1)))]
    assert not nb.matches(grown)  # densification: other tensors, other P
    with pytest.raises(RuntimeError, match="other tensors"):
        resolve_bucket(nb, lambda ps: GradBucket(ps, densify_points=10), grown)
    d = GradBucket([xyz])
    assert d.direct and d.matches([xyz, torch.nn.Parameter(torch.zeros(2), requires_grad=False)])
    assert resolve_bucket(None, None, [xyz]) is None
