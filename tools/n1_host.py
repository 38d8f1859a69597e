"""Host cost of the N > 1 step structure (measurement aid, round 6):

    python3 tools/n1_host.py [--steps 300] [--mode rccl|nodist|none] [--ar coalesce|c10d]

Builds bench.py's C3 language step as a PipelinedGraphStep with a GradBucket (mode rccl: a one-rank
RCCL group, the all-reduce launched eagerly between the backward and Adam graphs; nodist: the bucket
without a group; none: the N = 1 step) and prints, per step:
  wall        wall time per replay over the timed replays (run-ahead, as bench.py times it);
  host        the host's time inside replay() (if it approaches wall, the host paces the GPU);
  ar_host     the host's time inside the bucket's all_reduce (rccl only);
and the with-sync step (loss.item() after every replay).  --ar c10d routes the coalesced
{gradient, flag} all-reduce through the process group's allreduce_coalesced (one C++ call) instead
of torch.distributed's coalescing manager.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def arg(name, default):
    return sys.argv[sys.argv.index(name) + 1] if name in sys.argv else default


def main():
    import torch
    import torch.distributed as dist
    import bench
    from langsplat_amd import launch
    from langsplat_amd.distributed import GradBucket
    from langsplat_amd.pipeline import PipelinedGraphStep
    from langsplat_amd.synthetic import CONFIGS, make_cameras, make_gaussians
    steps = int(arg("--steps", "300"))
    mode = arg("--mode", "rccl")
    ar = arg("--ar", "coalesce")
    c = CONFIGS["C3"]
    P, W, H = c["P"], c["width"], c["height"]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if mode == "rccl":
        dist.init_process_group("nccl", rank=0, world_size=1, init_method=f"tcp://127.0.0.1:{launch.free_port()}")
    model = bench.Model(make_gaussians(P, seed=0).to(dev), include_feature=True)
    cam = make_cameras(1, W, H, device=dev)[0]
    bg = torch.zeros(3, device=dev)
    gen = torch.Generator().manual_seed(100)
    gt = torch.nn.functional.normalize(torch.randn((3, H, W), generator=gen), dim=0).to(dev)
    mask = (torch.rand((1, H, W), generator=gen) < 0.9).to(dev)
    optim = bench.AmdAdam([{"params": [model._language_feature], "lr": 0.0025, "name": "language_feature"}],
                          lr=0.0, eps=1e-15)
    bucket = GradBucket(model.trainable()) if mode in ("rccl", "nodist") else None
    ar_times = []
    if bucket is not None:
        orig = bucket.all_reduce

        def timed(*a, **k):
            t0 = time.perf_counter()
            orig(*a, **k)
            ar_times.append(time.perf_counter() - t0)
        if ar == "c10d" and mode == "rccl":
            pgc = dist.distributed_c10d._get_default_group()
            opts = dist.AllreduceCoalescedOptions()
            opts.reduceOp = dist.ReduceOp.AVG

            def c10d_ar(average=True, group=None, flag=None):
                bucket._attach()
                work = pgc.allreduce_coalesced([bucket.buffer(), flag.view(torch.float32)], opts)
                work.wait()
                bucket._divided_by = dist.get_world_size()
            orig = c10d_ar
        bucket.all_reduce = timed
    pg = PipelinedGraphStep(lambda: bench.render(cam, model, bench.Pipe, bg, bench.Opt,
                                                 language_target=(gt, mask))["language_l1"],
                            model.trainable(), optim, bucket=bucket, model=model).capture()
    for _ in range(200):
        pg.replay()
    pg.synchronize()
    torch.cuda.synchronize()
    ar_times.clear()
    host = 0.0
    t0 = time.perf_counter()
    for _ in range(steps):
        h = time.perf_counter()
        pg.replay()
        host += time.perf_counter() - h
    pg.synchronize()
    torch.cuda.synchronize()
    wall = 1e3 * (time.perf_counter() - t0) / steps
    ar_ms = 1e3 * sum(ar_times) / max(1, len(ar_times))
    t0 = time.perf_counter()
    for _ in range(steps):
        pg.replay().item()
    torch.cuda.synchronize()
    synced = 1e3 * (time.perf_counter() - t0) / steps
    ok = pg.check()
    coll = float("nan")
    if mode == "rccl":  # the collective alone: eager, its GPU time per call by events on the stream
        part = torch.zeros((3 * P + 1,), device=dev)  # the deferred tail's partials + skip word
        b2 = GradBucket(model.trainable())
        for _ in range(10):
            b2.all_reduce_partials(part)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(50):
            b2.all_reduce_partials(part)
        e1.record()
        torch.cuda.synchronize()
        coll = e0.elapsed_time(e1) / 50
    print(f"n1_host: mode {mode} ar {ar}  wall {wall:.4f} ms/step  host {1e3 * host / steps:.4f}  "
          f"ar_host {ar_ms:.4f}  synced {synced:.4f}  collective alone {coll:.4f}  check {ok}", flush=True)
    if dist.is_initialized():
        torch.cuda.synchronize()
        from langsplat_amd import rccl
        rccl.destroy_default()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
