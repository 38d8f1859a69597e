"""_lsr_autograd (langsplat_amd/csrc/lsr_autograd.cpp), host side: a parameter's cached AccumulateGrad
node is seen and released while an old autograd graph (train.py:92-108 keeps the previous iteration's
loss alive) still holds it; the next graph gets its own node, and both graphs still accumulate into
the same .grad.  The stream binding itself needs a GPU (tests/test_gpu_capture_safety.py)."""
import pytest
import torch

from langsplat_amd import _native
from langsplat_amd.graph import release_stale_accumulators


def test_release_with_a_live_graph():
    A = _native.autograd_helper()
    p = torch.nn.Parameter(torch.arange(4.0))
    assert not A.release_accumulator(p)          # no graph yet: nothing cached
    old = (p * 2.0).sum()                        # the previous iteration's loss, still alive
    n_old = old.grad_fn.next_functions[0][0]
    assert release_stale_accumulators([p]) == 1
    new = (p * 3.0).sum()
    n_new = new.grad_fn.next_functions[0][0]
    assert n_new is not n_old                     # a fresh node for the new graph
    new.backward()
    assert torch.equal(p.grad, torch.full((4,), 3.0))
    old.backward()                                # the old graph's node still targets p
    assert torch.equal(p.grad, torch.full((4,), 5.0))


def test_release_refuses_non_leaves():
    A = _native.autograd_helper()
    p = torch.nn.Parameter(torch.ones(3))
    with pytest.raises(ValueError):
        A.release_accumulator(p * 2.0)
    with pytest.raises(TypeError):
        A.release_accumulator([1, 2])
    frozen = torch.ones(3)
    assert release_stale_accumulators([frozen]) == 0  # frozen parameters are skipped
