"""Oracle restatement of GaussianModel's activations vs torch itself.

The fused path (include/lsr.h lsr_raw_flags) activates raw parameters inside the kernels with
the oracle's operation sequence (lso_activate), so it is bit-exact against the oracle; these
tests pin that restatement to torch's own sigmoid / exp / F.normalize / language normalisation
(scene/gaussian_model.py:33-41, gaussian_renderer/__init__.py:87) and to torch autograd for the
backward.  CPU only.
"""
import numpy as np
import torch

from oracle import oracle


def _raw(P=4096, seed=0):
    g = torch.Generator().manual_seed(seed)
    op = torch.randn((P, 1), generator=g) * 6.0
    sc = torch.rand((P, 3), generator=g) * 12.0 - 10.0
    rot = torch.randn((P, 4), generator=g)
    lang = torch.randn((P, 3), generator=g)
    # edges: saturated logits, tiny / huge log-scales, zero quaternion, zero language vector
    op[:4, 0] = torch.tensor([-100.0, 100.0, 0.0, -87.5])
    sc[0] = torch.tensor([-100.0, 80.0, 0.0])
    rot[0] = 0.0
    rot[1] = torch.tensor([1e-20, 0.0, 0.0, 0.0])
    lang[0] = 0.0
    return op, sc, rot, lang


def test_activation_matches_torch():
    op, sc, rot, lang = _raw()
    a_op, a_sc, a_rot, a_lang = oracle.activate(oracle.RAW_ALL, op, sc, rot, lang)
    ref_op = torch.sigmoid(op).numpy()
    ref_sc = torch.exp(sc).numpy()
    ref_rot = torch.nn.functional.normalize(rot).numpy()
    ref_lang = (lang / (lang.norm(dim=-1, keepdim=True) + 1e-9)).numpy()
    # a few ulp (the exp restatement is not correctly rounded); denormal results flush to 0
    np.testing.assert_allclose(a_op, ref_op, rtol=6e-7, atol=1e-37)
    np.testing.assert_allclose(a_sc, ref_sc, rtol=6e-7, atol=1e-37)
    np.testing.assert_allclose(a_rot, ref_rot, rtol=4e-7, atol=1e-37)
    np.testing.assert_allclose(a_lang, ref_lang, rtol=4e-7, atol=1e-37)
    assert np.all(a_rot[0] == 0.0) and np.all(a_lang[0] == 0.0)


def test_activation_flags_select_inputs():
    op, sc, rot, lang = _raw(P=64, seed=1)
    a_op, a_sc, a_rot, a_lang = oracle.activate(oracle.RAW_SCALES, op, sc, rot, lang)
    assert np.all(a_op == 0) and np.all(a_rot == 0) and np.all(a_lang == 0)
    np.testing.assert_allclose(a_sc, torch.exp(sc).numpy(), rtol=6e-7, atol=1e-37)


def test_activation_backward_matches_autograd():
    op, sc, rot, lang = _raw(P=2048, seed=2)
    sc = sc.clamp(max=5.0)
    leaves = [t.clone().requires_grad_(True) for t in (op, sc, rot, lang)]
    outs = [torch.sigmoid(leaves[0]), torch.exp(leaves[1]), torch.nn.functional.normalize(leaves[2]),
            leaves[3] / (leaves[3].norm(dim=-1, keepdim=True) + 1e-9)]
    g = torch.Generator().manual_seed(5)
    gs = [torch.randn(o.shape, generator=g) for o in outs]
    torch.autograd.backward(outs, gs)
    mine = oracle.activate_backward(oracle.RAW_ALL, (op, sc, rot, lang), gs)
    for name, m, leaf in zip(("opacity", "scales", "rotations", "language"), mine, leaves):
        ref = leaf.grad.numpy()
        # zero vectors: torch's norm backward masks to 0 and so does the restatement
        np.testing.assert_allclose(m, ref, rtol=2e-5, atol=1e-6 * np.abs(ref).max(), err_msg=name)
