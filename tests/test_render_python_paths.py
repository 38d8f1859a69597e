"""render()'s Python-side alternatives on the CPU.

render.eval_sh is the restatement render() runs under pipe.convert_SHs_python
(gaussian_renderer/__init__.py:72-80); it must reproduce utils/sh_utils.py:eval_sh -- the values
and, through the +0.5 / clamp_min(0) of :80, the autograd gradients w.r.t. the coefficients and
the unnormalised view direction -- as recorded in tests/golden/sh_eval.npz (written by the
reference's own eval_sh, tests/golden/make_golden.py).  tests/test_gpu_render_paths.py runs the
switch end to end on the GPU.
"""
import os

import numpy as np
import pytest
import torch

from langsplat_amd.render import eval_sh

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def sh_gold():
    return np.load(os.path.join(GOLD, "sh_eval.npz"))


@pytest.mark.parametrize("deg", [0, 1, 2, 3])
def test_render_eval_sh_matches_reference_values_and_grads(sh_gold, deg):
    sh = torch.tensor(sh_gold[f"deg{deg}_sh"], dtype=torch.float64, requires_grad=True)  # (N, 3, 16)
    dirs_raw = torch.tensor(sh_gold[f"deg{deg}_dirs_raw"], dtype=torch.float64, requires_grad=True)
    dirs = dirs_raw / dirs_raw.norm(dim=1, keepdim=True)  # gaussian_renderer/__init__.py:77
    val = eval_sh(deg, sh, dirs)
    np.testing.assert_allclose(val.detach().numpy(), sh_gold[f"deg{deg}_value"], rtol=1e-12, atol=1e-14)
    rgb = torch.clamp_min(val + 0.5, 0.0)  # gaussian_renderer/__init__.py:80
    np.testing.assert_allclose(rgb.detach().numpy(), sh_gold[f"deg{deg}_rgb"], rtol=1e-12, atol=1e-14)
    (rgb * torch.tensor(sh_gold[f"deg{deg}_grad_out"])).sum().backward()
    np.testing.assert_allclose(sh.grad.numpy(), sh_gold[f"deg{deg}_grad_sh"], rtol=1e-12, atol=1e-14)
    gd = dirs_raw.grad.numpy() if dirs_raw.grad is not None else np.zeros_like(sh_gold[f"deg{deg}_dirs_raw"])
    np.testing.assert_allclose(gd, sh_gold[f"deg{deg}_grad_dirs_raw"], rtol=1e-10, atol=1e-13)


def test_render_eval_sh_float32_close_to_reference(sh_gold):
    """render() runs eval_sh in fp32 on the model's tensors: within fp32 rounding of the reference."""
    sh = torch.tensor(sh_gold["deg3_sh"], dtype=torch.float32)
    dirs_raw = torch.tensor(sh_gold["deg3_dirs_raw"], dtype=torch.float32)
    dirs = dirs_raw / dirs_raw.norm(dim=1, keepdim=True)
    np.testing.assert_allclose(eval_sh(3, sh, dirs).numpy(), sh_gold["deg3_value"], rtol=1e-5, atol=2e-6)
