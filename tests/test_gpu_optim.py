"""langsplat_amd.optim.Adam (one HIP kernel per parameter) vs torch.optim.Adam.

Same algorithm, scalar handling and (explicit) FMAs as torch's single-tensor Adam; agreement is
to float rounding: rtol 2e-6 with an absolute floor of 1e-6 x max|value| for entries near zero,
after several steps with a changing learning rate."""
import pytest
import torch

from langsplat_amd.optim import Adam

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("shape", [(1000, 3), (4097,), (33, 1, 3)])
def test_adam_matches_torch(shape):
    g = torch.Generator().manual_seed(sum(shape))
    p0 = torch.randn(shape, generator=g)
    a = p0.clone().to(DEV).requires_grad_(True)
    b = p0.clone().to(DEV).requires_grad_(True)
    mine = Adam([{"params": [a], "lr": 0.01, "name": "x"}], lr=0.0, eps=1e-15)
    ref = torch.optim.Adam([{"params": [b], "lr": 0.01, "name": "x"}], lr=0.0, eps=1e-15, foreach=False)
    for it in range(6):
        gr = torch.randn(shape, generator=g).to(DEV)
        a.grad = gr.clone()
        b.grad = gr.clone()
        for grp in mine.param_groups + ref.param_groups:
            grp["lr"] = 0.01 * (0.7 ** it)  # update_learning_rate-style schedule
        mine.step()
        ref.step()
        sm, sr = mine.state[a], ref.state[b]
        for x, y in ((a.detach(), b.detach()), (sm["exp_avg"], sr["exp_avg"]), (sm["exp_avg_sq"], sr["exp_avg_sq"])):
            torch.testing.assert_close(x, y, rtol=2e-6, atol=1e-6 * float(y.abs().max()))
        assert float(sm["step"]) == float(sr["step"]) == it + 1
