#!/usr/bin/env python3
"""W ranks of the xgmi all-reduce sharing ONE GPU (gloo process group): per call, per rank, the
wall time, whether the result is the exact sum and whether a peer wait timed out (error word).
Tells a co-scheduling stall (every rank times out, results partly reduced) from a wrong sum
(no timeout, values off).

    python scripts/probe_xgmi_world.py --world 8 [--n 1048576] [--calls 3] [--blocks B]
"""
import argparse
import json
import os
import socket
import sys
import time

import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, n, calls, blocks, selftest, wire, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK='0', DQN_DIST_BACKEND='gloo')
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from dist_dqn_amd.parallel import init_distributed
    from dist_dqn_amd.parallel.xgmi import XgmiAllReduce
    out = {'rank': rank, 'calls': []}
    try:
        ctx = init_distributed(None, device='cuda')
        x = XgmiAllReduce(ctx, n, wire)
        if selftest:                     # XgmiAllReduce.self_test as the tests call it (both channels)
            t0 = time.perf_counter()
            out['self_test'] = bool(x.self_test(n))
            out['self_test_s'] = round(time.perf_counter() - t0, 3)
            out['self_test_log'] = x.self_test_log
        idx = torch.arange(n, device='cuda', dtype=torch.float32)
        nb = blocks or x.blocks_for(n)
        out['blocks'] = nb
        for c in range(calls):
            t = (idx % 7) + (rank + 1) * (c + 1)
            expect = world * (idx % 7) + (c + 1) * world * (world + 1) / 2
            dist.barrier()
            t0 = time.perf_counter()
            x.allreduce(t, channel=0, blocks=nb)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            bad = int((t != expect).sum())
            out['calls'].append({'s': round(dt, 4), 'wrong': bad, 'err_word': int(not x.check()),
                                 'seq': [int(v) for v in x.channels[0].seq_err[:4].tolist()]})
        dist.barrier()
        x.close()
        dist.destroy_process_group()
    except BaseException as e:  # noqa: BLE001
        out['exc'] = repr(e)
    q.put(json.dumps(out))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--world', type=int, default=8)
    ap.add_argument('--n', type=int, default=1 << 20)
    ap.add_argument('--calls', type=int, default=3)
    ap.add_argument('--blocks', type=int, default=0)
    ap.add_argument('--timeout', type=int, default=120)
    ap.add_argument('--selftest', type=int, default=0)
    ap.add_argument('--wire', default='fp32')
    a = ap.parse_args()
    ctx = mp.get_context('spawn')
    q = ctx.SimpleQueue()
    port = _free_port()
    ps = [ctx.Process(target=_rank, args=(r, a.world, port, a.n, a.calls, a.blocks, a.selftest, a.wire, q)) for r in range(a.world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=a.timeout)
    hung = [i for i, p in enumerate(ps) if p.is_alive()]
    for i in hung:
        ps[i].kill()
    res = []
    while not q.empty():
        res.append(json.loads(q.get()))
    res.sort(key=lambda d: d['rank'])
    print(json.dumps({'world': a.world, 'n': a.n, 'hw_queues': os.environ.get('GPU_MAX_HW_QUEUES'),
                      'hung': hung, 'ranks': res}))


if __name__ == '__main__':
    main()
