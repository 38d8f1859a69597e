"""Probe: do the two branches of a captured HIP graph run concurrently?  Two forked streams each
sleep ~1 ms inside one graph; a replay near 1 ms means concurrent branches, near 2 ms serialised."""
import time

import torch


def main():
    s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()
    cycles = 2_000_000
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s0):
        ev = torch.cuda.Event()
        ev.record(s0)
        s1.wait_event(ev)
        torch.cuda._sleep(cycles)
        with torch.cuda.stream(s1):
            torch.cuda._sleep(cycles)
        s0.wait_stream(s1)
    for mode in ("one", "graph"):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(10):
            if mode == "one":
                torch.cuda._sleep(cycles)
            else:
                g.replay()
        torch.cuda.synchronize()
        print(mode, f"{(time.perf_counter() - t) / 10 * 1e3:.3f} ms")


if __name__ == "__main__":
    main()
