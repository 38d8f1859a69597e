"""Engine clock vs the pipelined step's speed level (measurement aid):

    python3 tools/clock_probe.py

bench.py's PipelinedGraphStep at C3, REPS reps of STEPS replays (drained, then a short pause, between
reps).  Every EVERY replays a one-wave probe kernel (include/lsr.h lsr_debug_clock_probe) on a third
stream measures the engine clock over ~20 us while the step's kernels run: 100 x (shader-clock ticks)
/ (100 MHz ticks).  Prints each rep's wall time per step beside the mean / min probe clock, then the
correlation of the two over the reps.
"""
import ctypes
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from langsplat_amd import _native
    from langsplat_amd.pipeline import PipelinedGraphStep
    from langsplat_amd.synthetic import CONFIGS, make_cameras, make_gaussians
    steps = int(os.environ.get("CP_STEPS", "300"))
    reps = int(os.environ.get("CP_REPS", "10"))
    every = int(os.environ.get("CP_EVERY", "10"))
    pause = float(os.environ.get("CP_PAUSE", "0.02"))
    c = CONFIGS["C3"]
    P, W, H = c["P"], c["width"], c["height"]
    dev = torch.device("cuda", 0)
    model = bench.Model(make_gaussians(P, seed=0).to(dev), include_feature=True)
    cam = make_cameras(1, W, H, device=dev)[0]
    bg = torch.zeros(3, device=dev)
    gen = torch.Generator().manual_seed(100)
    gt = torch.nn.functional.normalize(torch.randn((3, H, W), generator=gen), dim=0).to(dev)
    mask = (torch.rand((1, H, W), generator=gen) < 0.9).to(dev)
    optim = bench.AmdAdam([{"params": [model._language_feature], "lr": 0.0025, "name": "language_feature"}],
                          lr=0.0, eps=1e-15)
    pg = PipelinedGraphStep(lambda: bench.render(cam, model, bench.Pipe, bg, bench.Opt,
                                                 language_target=(gt, mask))["language_l1"],
                            [model._language_feature], optim, model=model).capture()
    lib = _native.load()
    probe_stream = torch.cuda.Stream(dev)
    nprobe = steps // every
    buf = torch.zeros((nprobe, 4), dtype=torch.int64, device=dev)
    for _ in range(20):
        pg.replay()
    pg.synchronize()
    torch.cuda.synchronize()
    rows = []
    for rep in range(reps):
        time.sleep(pause)
        buf.zero_()
        t0 = time.perf_counter()
        for k in range(steps):
            pg.replay()
            if k % every == every // 2 and k // every < nprobe:
                with torch.cuda.stream(probe_stream):
                    _native._check(lib.lsr_debug_clock_probe(ctypes.c_void_p(buf[k // every].data_ptr()),
                                                             ctypes.c_void_p(probe_stream.cuda_stream)),
                                   "lsr_debug_clock_probe")
        pg.synchronize()
        torch.cuda.synchronize()
        wall = 1e3 * (time.perf_counter() - t0) / steps
        b = buf.cpu().tolist()
        mhz = [100.0 * (x[3] - x[1]) / (x[2] - x[0]) for x in b if x[2] > x[0]]
        rows.append((wall, statistics.mean(mhz), min(mhz), max(mhz)))
        print(f"rep {rep:2d}: {wall:.4f} ms/step  clock mean {rows[-1][1]:7.1f} min {rows[-1][2]:7.1f} "
              f"max {rows[-1][3]:7.1f} MHz  ({len(mhz)} probes)", flush=True)
    w = [r[0] for r in rows]
    m = [r[1] for r in rows]
    mw, mm = statistics.mean(w), statistics.mean(m)
    cov = sum((a - mw) * (b - mm) for a, b in zip(w, m))
    den = (sum((a - mw) ** 2 for a in w) * sum((b - mm) ** 2 for b in m)) ** 0.5
    print(f"correlation(step time, mean clock) over {len(rows)} reps: {cov / den if den else float('nan'):.3f}")


if __name__ == "__main__":
    main()
