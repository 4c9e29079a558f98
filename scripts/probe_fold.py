"""Probe: the fused fc forward + scalar head launch (csrc/kernels/fc_head.hip) of the flagship
step, per-block phase stamps (s_memrealtime, 100 MHz) relative to the launch's first block:

  0 start  1 h tile reduced  2 fold issued + stores complete  3 arrived (counter)
  tail (last arriver of a row group): 4 Q loaded  5 TD done  6 end

    python scripts/probe_fold.py [extra config flags...]

Prints one JSON line: min / median / max of each phase over the learner blocks, the tails'
phases, and the launch's span.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch
    from dist_dqn_amd.actors.device_actor import DeviceActor
    from dist_dqn_amd.config import preset
    from dist_dqn_amd.learner import Learner
    from dist_dqn_amd.models.network import Network
    from dist_dqn_amd.replay import DeviceReplay
    dev = torch.device('cuda', 0)
    cfg = preset('nature', 'Pong-v0', '--seed=0 --dtype=bf16 --replay_memory_capacity=65536 ' + ' '.join(sys.argv[1:]))
    net = Network.create_network(cfg, (84, 84, 4), 6, device=dev)
    rep = DeviceReplay(65536, (84, 84), 4, device=dev, prioritized=cfg.prioritized_replay)
    rep.fill_synthetic(65536, 6)
    actor = DeviceActor(net, rep, cfg, num_envs=4, steps_per_call=1, seed=3)
    learner = Learner(net, rep, cfg, use_graph=False, actor=actor if actor.can_fuse(cfg.minibatch_size) else None)
    ex = net.executor
    assert ex.fold_head and ex.can_fold_head(cfg.minibatch_size, 4)
    B = cfg.minibatch_size
    ninst = (3 if ex.double else 2) + (1 if learner.actor is not None else 0)
    nblk = ((B + 15) // 16) * (ex.HH // 16) * ninst
    ex.fold_prof = torch.zeros(nblk * 8, dtype=torch.int64, device=dev)
    out = {'blocks': nblk, 'instances': ninst}
    runs = []
    for it in range(20):
        ex.fold_prof.zero_()
        learner.step()
        torch.cuda.synchronize()
        p = ex.fold_prof.view(nblk, 8).cpu().numpy().astype(np.float64)
        if it >= 5:
            runs.append(p)
    ex.fold_prof = None
    nl = ((B + 15) // 16) * (ex.HH // 16) * (3 if ex.double else 2)
    stats = {k: [] for k in ('gemm', 'fold', 'arrive', 'start')}
    tails = []
    spans = []
    for p in runs:
        valid = p[:, 0] > 0
        t0 = p[valid, 0].min()
        lp = p[:nl]
        stats['start'] += list((lp[:, 0] - t0) / 100.0)
        stats['gemm'] += list((lp[:, 1] - t0) / 100.0)
        stats['fold'] += list((lp[:, 2] - t0) / 100.0)
        stats['arrive'] += list((lp[:, 3] - t0) / 100.0)
        for row in lp[lp[:, 6] > 0]:
            tails.append([(row[i] - t0) / 100.0 for i in (3, 4, 5, 6)])
        spans.append((p[valid].max() - t0) / 100.0)
    q = lambda v: [round(float(np.min(v)), 2), round(float(np.median(v)), 2), round(float(np.max(v)), 2)]
    out['learner_blocks_us'] = {k: q(v) for k, v in stats.items()}
    out['tails_us'] = {'arrive/qload/td/end': [round(float(x), 2) for x in np.median(np.array(tails), 0)]} if tails else {}
    out['span_us'] = q(spans)
    print(json.dumps(out))


if __name__ == '__main__':
    main()
