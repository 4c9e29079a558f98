"""Do two HIP graphs replayed on two streams overlap, with per-iteration lagged
event dependencies (actor graph i after learner snapshot i-1; snapshot i after
actor graph i)? Compares: serial (one stream), and two streams + events."""
import time

import torch

dev = torch.device('cuda', 0)
torch.cuda.set_device(dev)
CYC = 3000


def graph(n, stream):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(stream):
        torch.cuda._sleep(10)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=stream):
            for _ in range(n):
                torch.cuda._sleep(CYC)
    return g


s_l, s_a = torch.cuda.Stream(), torch.cuda.Stream()
gl, ga, gs = graph(10, s_l), graph(3, s_a), graph(1, s_l)   # learner, actor, snapshot copy
torch.cuda.synchronize()


def serial(iters):
    with torch.cuda.stream(s_l):
        for _ in range(iters):
            ga.replay(); gl.replay(); gs.replay()


ev_act = [torch.cuda.Event() for _ in range(2)]
ev_snap = [torch.cuda.Event() for _ in range(2)]


def overlapped(iters):
    for i in range(iters):
        p, q = i % 2, (i + 1) % 2
        with torch.cuda.stream(s_a):
            if i > 0:
                s_a.wait_event(ev_snap[q])
            ga.replay()
            ev_act[p].record(s_a)
        with torch.cuda.stream(s_l):
            gl.replay()
            s_l.wait_event(ev_act[p])
            gs.replay()
            ev_snap[p].record(s_l)


for name, fn in (('serial', serial), ('overlap', overlapped), ('serial', serial), ('overlap', overlapped)):
    fn(5)
    torch.cuda.synchronize()
    t = time.perf_counter()
    fn(200)
    torch.cuda.synchronize()
    print('%-8s %.1f us/iter' % (name, (time.perf_counter() - t) / 200 * 1e6))
