"""HBM reference rates on this box (torch kernels, CUDA events over back-to-back launches): a
copy of R MB (R read + R written), a read-only reduction and a fill, at the byte counts of the
flagship (~34 MB moved) and Rainbow (~200 MB) optimizer launches. The optimizer's achieved rate
is judged against these, not against the 8 TB/s datasheet peak.

    python scripts/probe_hbm.py
"""
import json

import torch


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000.0 / iters


def main():
    dev = torch.device('cuda', 0)
    out = {}
    for mb in (17, 100):
        n = mb * (1 << 20) // 4
        x = torch.randn(n, device=dev)
        y = torch.empty_like(x)
        s = torch.empty(1, device=dev)
        us = timeit(lambda: y.copy_(x))
        out['copy_%dMB' % mb] = {'us': round(us, 2), 'TBps': round(2 * mb * 1.048576e6 / us / 1e6, 2)}
        us = timeit(lambda: torch.sum(x, dim=0, out=s))
        out['read_%dMB' % mb] = {'us': round(us, 2), 'TBps': round(mb * 1.048576e6 / us / 1e6, 2)}
        us = timeit(lambda: y.fill_(1.0))
        out['write_%dMB' % mb] = {'us': round(us, 2), 'TBps': round(mb * 1.048576e6 / us / 1e6, 2)}
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
