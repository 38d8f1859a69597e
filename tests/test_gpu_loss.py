"""Masked L1 and ground-truth decode kernels vs torch.

Reference formulation: l1_loss(pred * mask, gt * mask) with l1_loss = torch.abs(a - b).mean()
(train.py:98, utils/loss_utils.py:17-18) evaluated by torch on the same GPU tensors.  The loss
value differs only by summation order (rtol 1e-6); the gradient is bit-identical.  The decode
follows Camera.get_language_feature (scene/cameras.py:63-92), restated in torch below.
"""
import numpy as np
import pytest
import torch

from langsplat_amd import _native
from langsplat_amd.loss import LanguageFeatureCache, decode_language_feature, masked_l1_loss

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _torch_l1(pred, gt, mask):
    return torch.abs(pred * mask - gt * mask).mean()


@pytest.mark.parametrize("H,W,mask_kind", [(64, 96, "bool"), (45, 67, "bool"), (64, 96, "float"),
                                           (1080, 1920, "bool"), (7, 5, "float")])
def test_masked_l1_matches_torch(H, W, mask_kind):
    g = torch.Generator().manual_seed(H * 1000 + W)
    pred = torch.randn((3, H, W), generator=g).to(DEV).requires_grad_(True)
    gt = torch.nn.functional.normalize(torch.randn((3, H, W), generator=g), dim=0).to(DEV)
    m = torch.rand((1, H, W), generator=g) < 0.9
    mask = (m if mask_kind == "bool" else m.float()).to(DEV)
    pred.data[:, :2, :2] = gt[:, :2, :2]  # exact zeros of the difference: sign(0) = 0
    loss = masked_l1_loss(pred, gt, mask)
    loss.backward(torch.tensor(1.7, device=DEV))
    mine = pred.grad.clone()
    pred.grad = None
    ref = _torch_l1(pred, gt, mask)
    ref.backward(torch.tensor(1.7, device=DEV))
    torch.testing.assert_close(loss, ref.detach(), rtol=1e-6, atol=0)
    assert torch.equal(mine, pred.grad)


def test_masked_l1_is_deterministic():
    g = torch.Generator().manual_seed(3)
    pred = torch.randn((3, 540, 960), generator=g).to(DEV)
    gt = torch.randn((3, 540, 960), generator=g).to(DEV)
    mask = (torch.rand((1, 540, 960), generator=g) < 0.5).to(DEV)
    a = masked_l1_loss(pred, gt, mask)
    b = masked_l1_loss(pred, gt, mask)
    assert torch.equal(a, b)


def _reference_decode(seg_map, feature_map, level, H, W):
    """scene/cameras.py:63-92 on CPU tensors (the reference's own gather)."""
    y, x = torch.meshgrid(torch.arange(0, H), torch.arange(0, W), indexing="ij")
    x = x.reshape(-1, 1)
    y = y.reshape(-1, 1)
    seg = seg_map[:, y, x].squeeze(-1).long()
    mask = seg != -1
    point_feature1 = feature_map[seg[level:level + 1]].squeeze(0)
    mask = mask[level:level + 1].reshape(1, H, W)
    return point_feature1.reshape(H, W, -1).permute(2, 0, 1), mask


def test_decode_language_feature_matches_reference(tmp_path):
    g = torch.Generator().manual_seed(5)
    L, H, W, N, D = 4, 37, 53, 120, 3
    seg_map = torch.randint(-1, N, (L, H, W), generator=g).float()  # stored as float, .long() in the reference
    feature_map = torch.randn((N, D), generator=g)
    for level in range(L):
        f, m = decode_language_feature(seg_map.to(DEV), feature_map.to(DEV), level)
        rf, rm = _reference_decode(seg_map, feature_map, level, H, W)
        assert torch.equal(m.cpu(), rm)
        assert torch.equal(f.cpu(), rf.contiguous())
    # the per-view HBM cache reads the same files as Camera.get_language_feature
    np.save(tmp_path / "view0_s.npy", seg_map.numpy())
    np.save(tmp_path / "view0_f.npy", feature_map.numpy())

    class Cam:
        image_name, image_height, image_width = "view0", H, W

    cache = LanguageFeatureCache(DEV)
    f1, m1 = cache.get(Cam, str(tmp_path), 2)
    f2, _ = cache.get(Cam, str(tmp_path), 2)
    assert f1 is f2 and len(cache) == 1
    rf, rm = _reference_decode(seg_map, feature_map, 2, H, W)
    assert torch.equal(f1.cpu(), rf.contiguous()) and torch.equal(m1.cpu(), rm)


def test_masked_l1_stall_fallback_is_exact():
    """Spin limit 0: the last block recomputes every other block's sum from the inputs instead of
    waiting for it; the loss is bit-identical and the event is reported."""
    lib = _native.load()
    g = torch.Generator().manual_seed(4)
    pred = torch.randn((3, 720, 1280), generator=g).to(DEV)
    gt = torch.randn((3, 720, 1280), generator=g).to(DEV)
    mask = (torch.rand((1, 720, 1280), generator=g) < 0.9).to(DEV)
    a = masked_l1_loss(pred, gt, mask)
    torch.cuda.synchronize()
    lib.lsr_debug_scan_stalls()
    old = lib.lsr_debug_set_spin_limit(0)
    try:
        b = masked_l1_loss(pred, gt, mask)
        torch.cuda.synchronize()
        assert lib.lsr_debug_scan_stalls() == 1
    finally:
        lib.lsr_debug_set_spin_limit(old)
    assert torch.equal(a, b)


def test_decode_rejects_out_of_range_segment_ids():
    """feature_map[seg] in scene/cameras.py:75-84 raises IndexError for ids outside [-N, N)."""
    N, D = 10, 3
    feature_map = torch.randn((N, D)).to(DEV)
    for bad in (N, -N - 1):
        seg_map = torch.zeros((4, 8, 9), dtype=torch.int64)
        seg_map[1, 3, 4] = bad
        with pytest.raises(IndexError, match="outside"):
            decode_language_feature(seg_map.to(DEV), feature_map, 1)
    # other levels than the bad one decode (the reference only indexes the requested level)
    seg_map = torch.zeros((4, 8, 9), dtype=torch.int64)
    seg_map[1, 3, 4] = N
    f, m = decode_language_feature(seg_map.to(DEV), feature_map, 0)
    assert m.all() and torch.equal(f[:, 0, 0], feature_map[0])


def test_cache_crops_a_larger_segment_map_and_rejects_a_smaller_one(tmp_path):
    """scene/cameras.py:69-73 gathers seg_map[:, y, x] for y < H, x < W."""
    g = torch.Generator().manual_seed(6)
    L, N, D, H, W = 4, 50, 3, 20, 30
    big = torch.randint(-1, N, (L, H + 5, W + 7), generator=g)
    feature_map = torch.randn((N, D), generator=g)
    np.save(tmp_path / "v_s.npy", big.numpy())
    np.save(tmp_path / "v_f.npy", feature_map.numpy())

    class Cam:
        image_name, image_height, image_width = "v", H, W

    f, m = LanguageFeatureCache(DEV).get(Cam, str(tmp_path), 1)
    rf, rm = _reference_decode(big, feature_map, 1, H, W)
    assert torch.equal(f.cpu(), rf.contiguous()) and torch.equal(m.cpu(), rm)

    class Big:
        image_name, image_height, image_width = "v", H + 6, W

    with pytest.raises(IndexError):
        LanguageFeatureCache(DEV).get(Big, str(tmp_path), 1)
