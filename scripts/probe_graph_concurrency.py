"""Do independent branches of a captured HIP graph run concurrently on this
ROCm build, and what does a fork/join cost? Main chain of N0 short spin kernels,
side chain of N1; serial capture vs forked (side stream) capture."""
import time

import torch

dev = torch.device('cuda', 0)
torch.cuda.set_device(dev)


def run(fork, n0, n1, cyc):
    s0 = torch.cuda.Stream()
    s1 = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s0):
        torch.cuda._sleep(10)
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s0):
        if fork:
            s1.wait_stream(s0)
            with torch.cuda.stream(s1):
                for _ in range(n1):
                    torch.cuda._sleep(cyc)
            for _ in range(n0):
                torch.cuda._sleep(cyc)
            s0.wait_stream(s1)
        else:
            for _ in range(n0 + n1):
                torch.cuda._sleep(cyc)
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(200):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / 200 * 1e6


for cyc in (1000, 10000):
    for n0, n1 in ((16, 3), (1, 1), (8, 8)):
        print('spin %6d cyc  main %2d side %2d : serial %.1f us, forked %.1f us' % (
            cyc, n0, n1, run(False, n0, n1, cyc), run(True, n0, n1, cyc)))
