"""Per-workgroup timeline of the MSD depth sort's bucket kernel (measurement aid).

    python tools/bucket_timeline.py [C3]

Runs forwards with LSR_BUCKET_TIMELINE=1 and reads the {start, end, slot, keys} record each of
the 256 bucket workgroups wrote (include/lsr.h lsr_debug_bucket_timeline): span, CU fill, tail
and the longest buckets with their key counts and start times.
"""
import ctypes
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
os.environ.setdefault("LSR_BUCKET_TIMELINE", "1")

from langsplat_amd import _native  # noqa: E402
from langsplat_amd.rasterizer import GaussianRasterizationSettings  # noqa: E402
from langsplat_amd.synthetic import CONFIGS, activated_inputs, make_cameras, make_gaussians  # noqa: E402
from render_timeline import analyse, TICK_US  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
    c = CONFIGS[cfg]
    dev = torch.device("cuda")
    P, W, H = c["P"], c["width"], c["height"]
    g = make_gaussians(P, seed=0).to(dev)
    cam = make_cameras(1, W, H, device=dev)[0]
    st = GaussianRasterizationSettings(H, W, math.tan(cam.FoVx * 0.5), math.tan(cam.FoVy * 0.5),
                                       torch.zeros(3, device=dev), 1.0, cam.world_view_transform,
                                       cam.full_proj_transform, 3, cam.camera_center, False, False, True)
    with torch.no_grad():
        inp = activated_inputs(g)
    lib = _native.load()
    arr = (ctypes.c_uint32 * (8 * 256))()
    for it in range(4):  # the last iteration's records are read (warm caches)
        _native.rasterize_gaussians(st, inp["means3D"], inp["shs"], None, inp["language_feature_precomp"],
                                    inp["opacities"], inp["scales"], inp["rotations"], None)
        torch.cuda.synchronize()
        _native._check(lib.lsr_debug_bucket_timeline(arr, 256), "lsr_debug_bucket_timeline")
    v = list(arr)
    recs = [{"start": v[8 * b], "end": v[8 * b + 1], "tile": b, "slot": v[8 * b + 2], "keys": v[8 * b + 3],
             "ph": v[8 * b + 4:8 * b + 8], "batches": 0} for b in range(256)]
    keys = {r["tile"]: r["keys"] for r in recs}

    def phases(b):
        r = recs[b]
        if not r["ph"][2]:
            return f"keys {keys[b]}"
        t = [r["start"], r["ph"][3]] + list(r["ph"][:3]) + [r["end"]]
        d = [((t[i + 1] - t[i]) & 0xFFFFFFFF) * TICK_US for i in range(5)]
        return (f"keys {keys[b]}: load {d[0]:.1f}, pass0 {d[1]:.1f}, later passes {d[2]:.1f}, gathers {d[3]:.1f}, "
                f"offsets {d[4]:.1f} us")
    mb = os.environ.get("LSR_BUCKET_MARK_BASE")
    if mb in ("1", "2"):  # a library built with -DLSR_BUCKET_MARK_BASE=1 / 2
        def phases(b):  # noqa: F811
            r = recs[b]
            if not r["ph"][2]:
                return f"keys {keys[b]}"
            t = [r["start"], r["ph"][0], r["ph"][1], r["ph"][2], r["ph"][3], r["end"]]
            d = [((t[i + 1] - t[i]) & 0xFFFFFFFF) * TICK_US for i in range(5)]
            if mb == "2":  # placed emission (the look-back before the sort): entries listed and ranked
                return (f"keys {keys[b]}: to pass0 {d[0]:.1f}, later passes {d[1]:.1f}, gathers {d[2]:.1f}, "
                        f"scan + list + rank {d[3]:.1f}, write {d[4]:.1f} us")
            return (f"keys {keys[b]}: to pass0 {d[0]:.1f}, later passes {d[1]:.1f}, gathers {d[2]:.1f}, "
                    f"scan + look-back {d[3]:.1f}, emission {d[4]:.1f} us")
    analyse(f"{cfg} depth bucket sort", recs, phases)
    full = [r for r in recs if r["ph"][2]]
    if full:
        import numpy as np
        a = np.array([[((r["ph"][3] - r["start"]) & 0xFFFFFFFF), ((r["ph"][1] - r["ph"][0]) & 0xFFFFFFFF),
                       ((r["ph"][2] - r["ph"][1]) & 0xFFFFFFFF), ((r["end"] - r["ph"][2]) & 0xFFFFFFFF),
                       r["keys"]] for r in full], dtype=np.float64)
        for lo, hi in ((0, 2000), (2000, 4000), (4000, 6000), (6000, 9000)):
            sel = a[(a[:, 4] >= lo) & (a[:, 4] < hi)]
            if len(sel):
                m = sel[:, :4].mean(0) * TICK_US
                print(f"  keys [{lo},{hi}): {len(sel)} buckets, mean load {m[0]:.1f}, later passes "
                      f"{m[1]:.1f}, gathers {m[2]:.1f}, offsets {m[3]:.1f} us")
    ks = sorted(keys.values(), reverse=True)
    print(f"  keys: total {sum(ks)}, max {ks[0]}, top-8 {ks[:8]}, non-empty {sum(1 for k in ks if k)}")
    starts = sorted(((r["start"] - min(x["start"] for x in recs)) & 0xFFFFFFFF) * TICK_US for r in recs)
    print(f"  start times (us): p10 {starts[25]:.1f}, p50 {starts[128]:.1f}, p90 {starts[230]:.1f}, "
          f"max {starts[-1]:.1f}")


if __name__ == "__main__":
    main()
