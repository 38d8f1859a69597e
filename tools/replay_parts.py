"""Host cost of the pieces of PipelinedGraphStep.replay() before its stream-A launch (measurement aid):

    python3 tools/replay_parts.py

Builds the C3 language step's pipelined graph (as bench.py does), then times each host operation
replay() performs before the step graph's launch, each in a loop of 2000 (median us per call), and
a ctypes round trip into liblsr.so for comparison with a native launch helper.
"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def per_call(fn, n=2000, reps=5):
    out = []
    for _ in range(reps):
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        out.append(1e6 * (time.perf_counter() - t0) / n)
    return statistics.median(out)


def main():
    import torch
    import bench
    from langsplat_amd import _native
    from langsplat_amd.graph import capture_key
    from langsplat_amd.pipeline import PipelinedGraphStep
    from langsplat_amd.synthetic import CONFIGS, make_cameras, make_gaussians
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
                            [model._language_feature], optim).capture()
    for _ in range(50):
        pg.replay()
    torch.cuda.synchronize()
    sa, sb = pg.streams
    ev = torch.cuda.Event()
    ev.record(sb)
    torch.cuda.synchronize()
    res = {}
    res["capture_key"] = per_call(lambda: capture_key(pg.model, pg.optimizer, pg.params))
    res["stream.wait_event"] = per_call(lambda: sa.wait_event(ev))
    def ctx():
        with torch.cuda.stream(sa):
            pass
    res["with torch.cuda.stream"] = per_call(ctx)
    res["optimizer.sync_lr"] = per_call(pg.optimizer.sync_lr)
    res["event.record(stream)"] = per_call(lambda: ev.record(sa))
    res["torch.cuda.current_stream"] = per_call(torch.cuda.current_stream)
    lib = _native.load()
    if lib is not None and hasattr(lib, "lsr_abi_version"):
        res["ctypes call (lsr_abi_version)"] = per_call(lib.lsr_abi_version)
    torch.cuda.synchronize()
    for k, v in res.items():
        print(f"replay_parts: {k:32s} {v:7.2f} us", flush=True)


if __name__ == "__main__":
    main()
