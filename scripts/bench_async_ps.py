"""Async parameter-server throughput (`--async_ps`, the reference's PS semantics,
`/root/reference/src/network.py:184-202`): rank 0 serves, ranks 1..W-1 run the HIP Nature-CNN
learner against it (push gradient, pull parameters + global_step). All ranks share ONE GPU here
(gloo for setup / p2p messages); `--transport xgmi` moves the data by one-sided peer access and
the control words through a host-shared page, `p2p` by `dist.isend/irecv`.

    python scripts/bench_async_ps.py --transport xgmi --workers 2 --steps 300

Prints one JSON line: PS updates/s (all workers), per-worker SGD steps/s, wall time.
"""
import argparse
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, transport, steps, q, pipeline=0, lowrank=1):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK='0', DQN_DIST_BACKEND='gloo')
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from dist_dqn_amd.config import preset
    from dist_dqn_amd.learner import Learner
    from dist_dqn_amd.models.network import Network
    from dist_dqn_amd.parallel import broadcast_state, init_distributed
    from dist_dqn_amd.parallel.async_ps import make_ps_client, make_ps_server
    from dist_dqn_amd.replay import DeviceReplay
    cfg = preset('nature', 'Pong-v0', '--dtype=bf16 --seed=5 --backend=hip --replay_memory_capacity=20000 '
                 '--async_ps --ps_transport=%s --ps_pipeline=%d --ps_lowrank=%d' % (transport, pipeline, lowrank))
    ctx = init_distributed(cfg, device='cuda')
    net = Network.create_network(cfg, (84, 84, 4), 6, num_replicas=world, device=ctx.device)
    broadcast_state(ctx, net)
    if rank == 0:
        srv = make_ps_server(ctx, net, cfg)
        t0 = time.perf_counter()
        n = srv.serve()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        # steady state: the native server's update timestamps (every 64th), middle half of the run
        mk = getattr(srv, 'marks', [])
        steady = None
        if len(mk) >= 8:
            i0, i1 = len(mk) // 4, 3 * len(mk) // 4
            steady = 64 * (i1 - i0) / (mk[i1] - mk[i0])
        q.put(('ps', n, el, steady))
        if hasattr(srv, 'close'):
            dist.barrier()
            srv.close()
    else:
        rep = DeviceReplay(20000, (84, 84), 4, device=ctx.device, seed=rank)
        rep.fill_synthetic(20000, 6, seed=rank)
        ps = make_ps_client(ctx, net.online.flat, cfg, network=net)
        ps.pull(net.online.flat, net.global_step)
        net.refresh_packed()
        ln = Learner(net, rep, cfg, ctx, ps_client=ps)
        for _ in range(5):
            ln.step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps - 5):
            ln.step()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        q.put(('worker', steps - 5, el))
        if transport == 'xgmi':
            ps.close()
            dist.barrier()
        else:
            ps.close()
    if transport != 'xgmi':
        dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--transport', choices=['p2p', 'xgmi'], default='xgmi')
    ap.add_argument('--workers', type=int, default=2)
    ap.add_argument('--steps', type=int, default=300, help='SGD steps (pushes) per worker')
    ap.add_argument('--pipeline', type=int, default=0, help='--ps_pipeline: take the previous push\'s answer, then push')
    ap.add_argument('--lowrank', type=int, default=1, help='--ps_lowrank: push the fc factors, not the fc gradient')
    args = ap.parse_args()
    import multiprocessing as mp
    ctx = mp.get_context('spawn')
    q = ctx.SimpleQueue()
    world = args.workers + 1
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, args.transport, args.steps, q, args.pipeline, args.lowrank)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=600)
    for p in procs:
        if p.is_alive():
            p.kill()
    res = []
    while not q.empty():
        res.append(q.get())
    ps = [r for r in res if r[0] == 'ps']
    steady = ps[0][3] if ps and len(ps[0]) > 3 else None
    wk = [r for r in res if r[0] == 'worker']
    out = {'transport': args.transport, 'workers': args.workers, 'steps_per_worker': args.steps,
           'pipeline': args.pipeline, 'lowrank': args.lowrank,
           'ps_updates': ps[0][1] if ps else None, 'ps_wall_s': round(ps[0][2], 3) if ps else None,
           'ps_updates_per_sec': round(ps[0][1] / ps[0][2], 1) if ps else None,
           # (the rate above includes the workers' start-up: replay fill, learner build, graph capture)
           'ps_updates_per_sec_steady': round(steady, 1) if steady else None,
           'worker_sgd_steps_per_sec': [round(n / el, 1) for _, n, el in wk],
           'exitcodes': [p.exitcode for p in procs], 'gpus': 1,
           'note': 'all ranks share one MI355X (gloo setup); the workers run the HIP Nature-CNN learner'}
    print(json.dumps(out), flush=True)
    sys.exit(0 if all(p.exitcode == 0 for p in procs) else 1)


if __name__ == '__main__':
    main()
