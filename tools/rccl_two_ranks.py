"""Probe: can two RCCL ranks share one GPU on this image?  (A 1-GPU box is all the builder gets; the
8-GPU node is the driver's.)  Run as `python tools/rccl_two_ranks.py` -- it starts its own 2 ranks
(langsplat_amd.launch).  Each rank: backend "nccl" on cuda:0, an eager SUM / AVG, the coalesced
{bucket, float-encoded flag} AVG of GradBucket.all_reduce(flag=), and the same captured into a HIP
graph and replayed.  Prints RCCL2_OK per rank, or the failure."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rank_main():
    import torch
    import torch.distributed as dist
    from langsplat_amd.distributed import GradBucket
    from langsplat_amd.graph import graph_capture
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", int(os.environ.get("LSR_PROBE_DEVICE", "0")))
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    t = torch.full((1024,), float(rank + 1), device=dev)
    dist.all_reduce(t)
    torch.cuda.synchronize()
    want = world * (world + 1) / 2
    assert torch.all(t == want), (rank, t[:4])
    P = 4096
    lang = torch.nn.Parameter(torch.zeros((P, 3), device=dev))
    b = GradBucket([lang])
    flag = torch.zeros((), dtype=torch.int32, device=dev)
    lang.grad = torch.full((P, 3), float(rank + 1), device=dev)
    b.all_reduce(average=True, flag=flag)
    torch.cuda.synchronize()
    assert torch.all(lang.grad == want / world) and int(flag.item()) == 0, rank
    out = torch.zeros((P, 3), device=dev)
    src = torch.zeros((P, 3), device=dev)
    fout = torch.zeros((), device=dev)
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side), graph_capture(g):
        lang.grad.copy_(src)
        b.all_reduce(average=True, flag=flag)
        out.copy_(lang.grad)
        fout.copy_(flag.view(torch.float32))
    torch.cuda.current_stream().wait_stream(side)
    for k in range(3):
        src.fill_(float((rank + 1) * (k + 1)))
        flag.fill_(0x3F800000 if (k == 1 and rank == world - 1) else 0)
        g.replay()
        torch.cuda.synchronize()
        assert torch.all(out == (k + 1) * want / world), (rank, k, out[0, 0].item())
        assert float(fout.item()) == (1.0 / world if k == 1 else 0.0), (rank, k, fout.item())
    dist.barrier()
    dist.destroy_process_group()
    print(f"RCCL2_OK rank {rank} of {world}", flush=True)


if __name__ == "__main__":
    if "RANK" in os.environ:
        rank_main()
    else:
        from langsplat_amd import launch
        sys.exit(launch.launch([os.path.abspath(__file__)], int(sys.argv[1]) if len(sys.argv) > 1 else 2))
