"""Per-workgroup timeline of the render kernels at a BASELINE config (measurement aid).

    python tools/render_timeline.py [C3] [--full]

The backward runs the bench's language-step variant (no colour gradient, no geometry gradients);
--full runs the variant with every gradient; --zero has the forward clear the language step's
gradient records (LSR_FWD_ZERO_GRAD_RECORDS, as the benched step does); --fwd-only skips the
backward (required with a measurement build whose forward leaves tiles unrendered).

Runs one forward + backward with LSR_RENDER_STATS=1 and reads the {start, end, tile, CU} record
every workgroup wrote (include/lsr.h lsr_debug_render_timeline).  Prints, per kernel, the span,
the summed workgroup time over (span x CUs) (how full the CUs were), the concurrency profile
(how much of the span ran below half / a quarter of the peak workgroup count: the tail), and the
longest workgroups with their start times.
"""
import math
import os
import sys
from collections import defaultdict

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("LSR_RENDER_STATS", "1")

from langsplat_amd import _native  # noqa: E402
from langsplat_amd.rasterizer import GaussianRasterizationSettings  # noqa: E402
from langsplat_amd.synthetic import CONFIGS, activated_inputs, make_cameras, make_gaussians  # noqa: E402

TICK_US = 0.01  # s_memrealtime: 100 MHz


MARKS = ("begin", "range", "barrier", "ids", "gather", "loaded")


def marks(ph):
    """The first batch's milestones, in us after the workgroup's start."""
    return " ".join(f"{n} {v * TICK_US:.1f}" for n, v in zip(MARKS, ph["first_marks"]))


def analyse(name, recs, info=None):
    recs = [(r["start"], r["end"], r["tile"], r["slot"], dict(r, b=b)) for b, r in enumerate(recs)
            if r["end"] != 0 or r["start"] != 0]
    if not recs:
        print(f"{name}: no records")
        return
    t0 = min(r[0] for r in recs)
    ev = []
    per_cu = defaultdict(float)
    dur = []
    phases = {}
    for r in recs:
        phases[r[2]] = r[4]
    blk = {}
    for s, e, tile, slot, r in recs:
        s, e = (s - t0) & 0xFFFFFFFF, (e - t0) & 0xFFFFFFFF
        ev.append((s, 1))
        ev.append((e, -1))
        per_cu[slot] += e - s
        dur.append((e - s, s, tile))
        blk[tile] = r["b"]
    span = max(e for e, _ in ev if _ == -1)
    ev.sort()
    cur = peak = 0
    prof = []
    last = 0
    for t, d in ev:
        prof.append((last, t, cur))
        cur += d
        peak = max(peak, cur)
        last = t
    below = {f: sum(b - a for a, b, c in prof if c < f * peak) for f in (0.5, 0.25)}
    busy = sum(d for d, _, _ in dur)
    ncu = len(per_cu)
    print(f"{name}: {len(recs)} workgroups on {ncu} CUs, span {span * TICK_US:.1f} us, "
          f"peak concurrency {peak} ({peak / max(ncu, 1):.1f}/CU)")
    print(f"  sum of workgroup time / (span x peak) = {busy / (span * peak):.3f}; "
          f"span below 1/2 peak: {below[0.5] / span:.3f}, below 1/4 peak: {below[0.25] / span:.3f}")
    tot = {k: sum(ph.get(k, 0) for ph in phases.values()) for k in ("load", "compact", "walk")}
    if sum(tot.values()):
        print("  phases summed over workgroups: " + ", ".join(f"{k} {100.0 * v / busy:.1f}%" for k, v in tot.items())
              + " of workgroup time")
    first = [(s, phases.get(tile)) for _, s, tile in dur
             if phases.get(tile) and phases[tile].get("batches") and "first_marks" in phases[tile]]
    if first:
        for lab, sel in (("starting < 2 us", [p for s, p in first if s * TICK_US < 2.0]),
                         ("starting later", [p for s, p in first if s * TICK_US >= 2.0])):
            if sel:
                m = [sum(p["first_marks"][k] for p in sel) / len(sel) for k in range(6)]
                print(f"  first batch, {len(sel)} workgroups {lab}: milestones " + marks({"first_marks": m}))
    dur.sort(reverse=True)
    mean = busy / len(dur)
    print(f"  workgroup time: mean {mean * TICK_US:.1f} us, max {dur[0][0] * TICK_US:.1f} us")
    for d, s, tile in dur[:5]:
        extra = info(tile) if info and tile >= 0 else ""
        ph = phases.get(tile)
        if ph and ph.get("batches") and "first_marks" in ph:
            extra += (f"\n        {ph['batches']} batches: load {ph['load'] * TICK_US:.1f} us (first "
                      f"{ph['first_load'] * TICK_US:.1f}; milestones " + marks(ph) + "), compact "
                      f"{ph['compact'] * TICK_US:.1f} us, walk {ph['walk'] * TICK_US:.1f} us")
        print(f"    tile {tile:6d} (workgroup {blk.get(tile, -1)}): {d * TICK_US:7.1f} us, starts at {s * TICK_US:6.1f} us "
              f"{extra}")


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    full = "--full" in sys.argv
    flags = _native.FWD_ZERO_GRAD_RECORDS if "--zero" in sys.argv else 0
    cfg = args[0] if args else "C3"
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
    gc = torch.randn((3, H, W), device=dev) / (3 * H * W)
    gl = torch.randn((3, H, W), device=dev) / (3 * H * W)
    tiles = ((W + 15) // 16) * ((H + 15) // 16)
    for it in range(3):  # the last iteration's records are read (warm caches)
        nr, color, lang, radii, geom, binning, image = _native.rasterize_gaussians(
            st, inp["means3D"], inp["shs"], None, inp["language_feature_precomp"], inp["opacities"],
            inp["scales"], inp["rotations"], None, flags=flags)
        torch.cuda.synchronize()
        fwd = _native.debug_render_timeline(0, tiles)
        if "--fwd-only" in sys.argv:
            continue
        _native.rasterize_gaussians_backward(st, inp["means3D"], inp["shs"], None, inp["language_feature_precomp"],
                                             inp["scales"], inp["rotations"], None, radii, gc if full else None, gl,
                                             nr, geom, binning, image, geometry=full)
        torch.cuda.synchronize()
        bwd = _native.debug_render_timeline(1, tiles)
    _native.debug_render_stats()
    lay = _native.state_layout(P, W, H, nr)
    gx, gy = (W + 15) // 16, (H + 15) // 16
    rng = image[lay["ranges"]:lay["ranges"] + 8 * tiles].view(torch.int32).view(tiles, 2).cpu().numpy()
    nc = image[lay["n_contrib"]:lay["n_contrib"] + 4 * W * H].view(torch.int32).cpu().numpy().reshape(H, W)
    fT = image[lay["final_T"]:lay["final_T"] + 4 * W * H].view(torch.float32).cpu().numpy().reshape(H, W)

    def info(tile):
        ty, tx = divmod(tile, gx)
        blk = nc[ty * 16:(ty + 1) * 16, tx * 16:(tx + 1) * 16]
        t = fT[ty * 16:(ty + 1) * 16, tx * 16:(tx + 1) * 16]
        return (f"list {int(rng[tile, 1] - rng[tile, 0])}, max n_contrib {int(blk.max())}, "
                f"saturated px {float((t < 1e-4).mean()):.2f}, mean final T {float(t.mean()):.2e}")
    analyse(f"{cfg} render forward", fwd, info)
    if "--fwd-only" not in sys.argv:
        nb = sum(1 for r in bwd if r["tile"] >= 0 and r["end"] != 0)
        analyse(f"{cfg} render backward", [r for r in bwd[:nb]], info)


if __name__ == "__main__":
    main()
