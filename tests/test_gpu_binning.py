"""Binning paths at the edges of the super-tile scheme, HIP vs the oracle (bit-exact forward).

The super-tile sort (lsr_binning.hip) is one 8-bit radix pass when the image has at most 256
super-tiles of 8 x 8 tiles (1080p: 135), and then takes the fused count kernel
(k_bin_count_fused: super-tile ranges straight from the scanned radix histogram); beyond 256
super-tiles it takes two passes and the k_super_ranges / k_seg_setup kernels.  Both must give the
oracle's per-tile lists, ranges and images bit for bit (up to 2188 super-tiles: a 140000 x 200
image).
"""
import math

import numpy as np
import pytest
import torch

from tests.scenes import settings_for
from tests.test_gpu_parity import check_backward, check_forward_exact
from langsplat_amd.synthetic import make_cameras

pytestmark = pytest.mark.gpu


def strip_scene(P, W, H, seed):
    """Gaussians spread over the whole field of view of a W x H camera at (0, 0, -4)."""
    g = torch.Generator().manual_seed(seed)
    cam = make_cameras(1, W, H)[0]
    tx, ty = math.tan(cam.FoVx * 0.5), math.tan(cam.FoVy * 0.5)
    d = 3.0 + torch.rand(P, generator=g) * 2.0
    u, v = torch.rand(P, generator=g) * 2 - 1, torch.rand(P, generator=g) * 2 - 1
    means = torch.stack([u * d * tx * 0.95, v * d * ty * 0.9, d - 4.0], 1)
    s = 0.04 * d / 4.0
    inp = dict(means3D=means, opacities=torch.rand((P, 1), generator=g) * 0.7 + 0.05,
               colors_precomp=torch.rand((P, 3), generator=g),
               language_feature_precomp=torch.nn.functional.normalize(torch.randn((P, 3), generator=g)),
               scales=s[:, None] * (0.5 + torch.rand((P, 3), generator=g)),
               rotations=torch.nn.functional.normalize(torch.randn((P, 4), generator=g)))
    return settings_for(cam, sh_degree=0), inp


@pytest.mark.parametrize("W,H,supers", [(2000, 250, 32), (8192, 72, 64), (33000, 64, 258), (140000, 200, 2188)])
def test_super_tile_counts(W, H, supers):
    st, inp = strip_scene(3000, W, H, seed=W + H)
    gx, gy = (W + 15) // 16, (H + 15) // 16
    assert ((gx + 7) // 8) * ((gy + 7) // 8) == supers
    run, std, ind, out = check_forward_exact(st, inp)
    assert out[0] > 0
    check_backward(st, inp, run, out)


@pytest.mark.parametrize("buckets", ["256", "512"])
def test_fused_emission_over_capacity(buckets, monkeypatch):
    """The depth sort's bucket workgroups write the super-tile entries themselves, into arrays of
    kFusedEntries (3) entries per Gaussian (lsr_internal.h).  A view whose Gaussians meet more
    super-tiles than that (E > 3 P) emits nothing there and takes k_emit_super after the host wait
    (its bucket bases from the 256 or 512 bucket totals).  Large Gaussians on a 1280x720 image: both
    the forward and the backward stay exact."""
    from tests.test_gpu_parity import state
    monkeypatch.setenv("LSR_MSD_BUCKETS", buckets)
    P, W, H = 300, 1280, 720
    g = torch.Generator().manual_seed(41)
    cam = make_cameras(1, W, H)[0]
    tx, ty = math.tan(cam.FoVx * 0.5), math.tan(cam.FoVy * 0.5)
    d = 3.0 + torch.rand(P, generator=g) * 2.0
    u, v = torch.rand(P, generator=g) * 2 - 1, torch.rand(P, generator=g) * 2 - 1
    means = torch.stack([u * d * tx * 0.8, v * d * ty * 0.8, d - 4.0], 1)
    inp = dict(means3D=means, opacities=torch.rand((P, 1), generator=g) * 0.3 + 0.05,
               colors_precomp=torch.rand((P, 3), generator=g),
               language_feature_precomp=torch.nn.functional.normalize(torch.randn((P, 3), generator=g)),
               scales=0.15 + 0.15 * torch.rand((P, 3), generator=g),
               rotations=torch.nn.functional.normalize(torch.randn((P, 4), generator=g)))
    st = settings_for(cam, sh_degree=0)
    run, std, ind, out = check_forward_exact(st, inp)
    assert state(out, P, W, H)["counters"][4] > 3 * P  # E: beyond the fused capacity
    check_backward(st, inp, run, out)


def dense_bucket_scene(seed=51):
    """1024 large Gaussians at one depth (one MSD bucket of the depth sort) over a 1280x720 view (60
    super-tiles), each meeting ~9-16 super-tiles: that bucket has more entries than one LDS list
    (kBucketCap = 8192), and more than 8192 within its one run of 1024 Gaussians; plus 7000 small
    Gaussians over depths 0.5..50, so E stays within the fused capacity (3 P)."""
    P1, P2, W, H = 1024, 7000, 1280, 720
    g = torch.Generator().manual_seed(seed)
    cam = make_cameras(1, W, H)[0]
    tx, ty = math.tan(cam.FoVx * 0.5), math.tan(cam.FoVy * 0.5)
    d = torch.cat([4.0 + torch.rand(P1, generator=g) * 1e-3,
                   torch.exp(torch.rand(P2, generator=g) * (math.log(50.0) - math.log(0.5)) + math.log(0.5))])
    P = P1 + P2
    u, v = torch.rand(P, generator=g) * 2 - 1, torch.rand(P, generator=g) * 2 - 1
    means = torch.stack([u * d * tx * 0.9, v * d * ty * 0.9, d - 4.0], 1)
    s = torch.cat([torch.full((P1,), 0.28), 0.01 * d[P1:] / 4.0])
    inp = dict(means3D=means, opacities=torch.rand((P, 1), generator=g) * 0.3 + 0.05,
               colors_precomp=torch.rand((P, 3), generator=g),
               language_feature_precomp=torch.nn.functional.normalize(torch.randn((P, 3), generator=g)),
               scales=s[:, None] * (0.8 + 0.4 * torch.rand((P, 3), generator=g)),
               rotations=torch.nn.functional.normalize(torch.randn((P, 4), generator=g)))
    return settings_for(cam, sh_degree=0), inp


def c3_scene():
    from langsplat_amd.synthetic import CONFIGS, activated_inputs, make_gaussians
    c = CONFIGS["C3"]
    g = make_gaussians(c["P"], seed=0)
    with torch.no_grad():
        inp = {k: v.contiguous() for k, v in activated_inputs(g).items()}
    cam = make_cameras(1, c["width"], c["height"])[0]
    return settings_for(cam, sh_degree=g.max_sh_degree), inp


@pytest.mark.parametrize("kind", ["dense_bucket", "c3"])
def test_placed_emission_equals_depth_order_emission(kind, monkeypatch):
    """Placed emission (the bucket sort writes every super-tile entry at its super-tile-major
    position, from the MSD histogram's scanned [super-tile][bucket] count table) against the
    depth-order emission it replaces (entries in depth order, then the binning's super-tile radix
    pass; LSR_PLACED=0): the same per-tile lists, ranges and images, bit for bit.  dense_bucket also
    takes the LDS sort's multi-list tail and place_runs' sub-lists."""
    from tests.test_gpu_parity import native_forward, state
    st, inp = dense_bucket_scene() if kind == "dense_bucket" else c3_scene()
    P = inp["means3D"].shape[0]
    W, H = st.image_width, st.image_height
    res = {}
    for placed in ("1", "0"):
        monkeypatch.setenv("LSR_PLACED", placed)
        _, _, out = native_forward(st, inp)
        s = state(out, P, W, H)
        s.update(nr=out[0], color=out[1].cpu().numpy(), lang=out[2].cpu().numpy(), radii=out[3].cpu().numpy())
        res[placed] = s
    a, b = res["1"], res["0"]
    E = int(a["counters"][4])
    assert E <= 3 * P  # within the fused capacity: the placed path ran
    if kind == "dense_bucket":
        assert E > 7000 + 8192
    assert a["nr"] == b["nr"] > 0
    for k in ("ranges", "point_list", "final_T", "n_contrib", "color", "lang", "radii", "counters"):
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)


def test_placed_emission_dense_bucket_oracle():
    """The dense-bucket scene (placed emission's multi-list and sub-list paths) against the oracle:
    forward bit-exact, backward within the parity tolerance."""
    st, inp = dense_bucket_scene()
    run, std, ind, out = check_forward_exact(st, inp)
    check_backward(st, inp, run, out)


_RADIX16_CHILD = """
from tests.scenes import scene
from tests.test_gpu_parity import check_backward, check_forward_exact
st, inp = scene(P=20000, W=640, H=360, seed=7, scale_range=(0.02, 0.15))
run, std, ind, out = check_forward_exact(st, inp)
assert out[0] > 0
check_backward(st, inp, run, out)
print("RADIX16_OK")
"""


def test_sixteen_key_radix_tiles_match_the_oracle():
    """Sorts above 16M keys use 16-key radix tiles (lsr_binning.hip radix_small), which no test
    scene reaches: a child process with LSR_RADIX_SMALL_MAX=0 (every sort on 16-key tiles) and
    LSR_DEPTH_LSD=1 (the depth order as LSD passes) renders a scene bit-exactly against the oracle."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, LSR_RADIX_SMALL_MAX="0", LSR_DEPTH_LSD="1",
               PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""))
    r = subprocess.run([sys.executable, "-c", _RADIX16_CHILD], cwd=root, env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0 and "RADIX16_OK" in r.stdout, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])


@pytest.mark.parametrize("placed", ["1", "0"])
@pytest.mark.parametrize("kind", ["dense_bucket", "c3"])
def test_512_msd_buckets_equal_256(kind, placed, monkeypatch):
    """Above 2M Gaussians the depth order's MSD pass makes 512 buckets (9-bit digits, lsr_binning.hip
    msd_digits) so the buckets stay within one LDS sort.  Forced at smaller P (LSR_MSD_BUCKETS=512):
    the same depth order, hence the same per-tile lists, ranges and images as the 256-bucket pass, bit
    for bit, with placed emission (its [super-tile][bucket] counts over 32 groups of 16 buckets) and
    with depth-order emission.  dense_bucket also puts one bucket beyond LDS (the global-memory sort,
    and placed emission's multi-list tail) beside the LDS buckets."""
    from tests.test_gpu_parity import native_forward, state
    st, inp = dense_bucket_scene() if kind == "dense_bucket" else c3_scene()
    P = inp["means3D"].shape[0]
    W, H = st.image_width, st.image_height
    monkeypatch.setenv("LSR_PLACED", placed)
    res = {}
    for nb in ("512", "256"):
        monkeypatch.setenv("LSR_MSD_BUCKETS", nb)
        _, _, out = native_forward(st, inp)
        s = state(out, P, W, H)
        s.update(nr=out[0], color=out[1].cpu().numpy(), lang=out[2].cpu().numpy(), radii=out[3].cpu().numpy())
        res[nb] = s
    a, b = res["512"], res["256"]
    assert a["nr"] == b["nr"] > 0
    for k in ("ranges", "point_list", "final_T", "n_contrib", "color", "lang", "radii", "counters"):
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)


def test_512_msd_buckets_oracle_and_stall_fallback(monkeypatch):
    """The 512-bucket depth order against the oracle (forward bit-exact, backward within the parity
    tolerance), then with every look-back on its stall path (spin limit 0: the bucket entry bases
    from the inputs, through the 9-bit bucket map): the same forward, and the stall reported."""
    from langsplat_amd import _native
    from tests.scenes import scene
    monkeypatch.setenv("LSR_MSD_BUCKETS", "512")
    st, inp = scene(P=40000, W=320, H=240, seed=9, sh_degree=1, scale_range=(0.01, 0.06))
    run, std, ind, out = check_forward_exact(st, inp)
    assert out[0] > 0
    check_backward(st, inp, run, out)
    lib = _native.load()
    torch.cuda.synchronize()
    lib.lsr_debug_scan_stalls()  # clear
    old = lib.lsr_debug_set_spin_limit(0)
    try:
        check_forward_exact(st, inp, run)
        torch.cuda.synchronize()
        assert lib.lsr_debug_scan_stalls() == 1
    finally:
        lib.lsr_debug_set_spin_limit(old)
