"""The oracle's upstream forms (oracle/lsr_oracle.c "Upstream forms") against its kernel form, on
the CPU at C1 (BASELINE.json configs[0]).

The kernels reproduce form 0 (FORM_KERNEL) bit for bit; forms 1 and 2 evaluate the published 3DGS
rasterizer's source expressions (literal power, correctly rounded exp, glm covariance products,
(f alpha) T blending) without and with nvcc-style contraction.  Their distance from form 0 is
therefore the measured distance of the HIP images from plausible upstream arithmetic.
tests/test_gpu_upstream_form.py measures it on the GPU at C1-C3; here the bounds are checked on the
oracle alone, with the geometry (radii, tile lists) allowed to differ only where a 1-ulp change of
the cut-offs decides.
"""
import numpy as np
import pytest
import torch

from langsplat_amd.synthetic import CONFIGS, activated_inputs, make_cameras, make_gaussians
from oracle import oracle
from tests.scenes import settings_for


def image_distance(a, b):
    d = np.abs(a.astype(np.float64) - b.astype(np.float64)).max(axis=0)
    return float(d.max()), int((d > 1e-5).sum())


def grad_distance(a, b):
    """(max relative error with the parity floor, entries beyond 1e-4) of a against b."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    floor = 1e-2 * (np.abs(b).max() if b.size else 0.0) + 1e-30
    r = np.abs(a - b) / (np.abs(b) + floor)
    return float(r.max()) if r.size else 0.0, int((r > 1e-4).sum())


@pytest.fixture(scope="module")
def c1_runs():
    c = CONFIGS["C1"]
    g = make_gaussians(c["P"], seed=0)
    cam = make_cameras(1, c["width"], c["height"])[0]
    st = settings_for(cam, sh_degree=3)
    with torch.no_grad():
        inp = {k: v.contiguous() for k, v in activated_inputs(g).items()}
    gen = torch.Generator().manual_seed(3)
    H, W = c["height"], c["width"]
    gc = torch.randn((3, H, W), generator=gen)
    gl = torch.randn((3, H, W), generator=gen)
    out = {}
    for form in (oracle.FORM_KERNEL, oracle.FORM_UPSTREAM, oracle.FORM_UPSTREAM_FMA):
        run = oracle.forward(st, form=form, **inp)
        out[form] = (run, run.backward(gc, gl))
    return out


@pytest.mark.parametrize("form", [1, 2])
def test_upstream_form_images_within_measured_bounds(c1_runs, form):
    base, _ = c1_runs[0]
    run, _ = c1_runs[form]
    assert run.num_rendered == base.num_rendered
    np.testing.assert_array_equal(run.radii, base.radii)
    np.testing.assert_array_equal(run.get("point_list"), base.get("point_list"))
    for img in ("color", "language"):
        mx, n = image_distance(getattr(run, img), getattr(base, img))
        assert mx <= 1e-2 and n <= 5, (img, mx, n)


@pytest.mark.parametrize("form", [1, 2])
def test_upstream_form_gradients_within_measured_bounds(c1_runs, form):
    _, gbase = c1_runs[0]
    _, g = c1_runs[form]
    for k in ("means2D", "colors_precomp", "opacities", "means3D", "language_feature_precomp", "shs", "scales",
              "rotations"):
        mx, n = grad_distance(gbase[k], g[k])
        assert n <= max(2, 5e-5 * g[k].size) and mx <= 0.1, (k, mx, n)


def test_forms_differ_and_kernel_form_is_default(c1_runs):
    """The upstream forms are a different arithmetic (not silently form 0), and form 0 is what
    oracle.forward runs by default (the GPU parity contract)."""
    base, _ = c1_runs[0]
    assert c1_runs[1][0].form == 1 and base.form == 0
    assert not np.array_equal(c1_runs[1][0].color, base.color)
    assert not np.array_equal(c1_runs[2][0].color, base.color)
