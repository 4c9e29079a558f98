"""Run-to-run determinism of the HIP learner: the same seeded config twice (graph replay,
6 steps), per-tensor max |diff| of the parameters. The conv weight gradients sum their
M-chunk partials with fp32 atomics, so their last bits can depend on arrival order.
    python scripts/probe_determinism.py [extra config flags]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dist_dqn_amd.config import preset  # noqa: E402
from dist_dqn_amd.learner import Learner  # noqa: E402
from dist_dqn_amd.models.network import Network  # noqa: E402
from dist_dqn_amd.replay import DeviceReplay  # noqa: E402

extra = ' '.join(sys.argv[1:])
dev = torch.device('cuda', 0)


def run(fuse):
    cfg = preset('nature', 'Pong-v0', '--seed=3 --backend=hip --dtype=bf16 --replay_memory_capacity=4096 '
                 '--fuse_sampling=%d %s' % (fuse, extra))
    net = Network.create_network(cfg, (84, 84, 4), 6, device=dev)
    rep = DeviceReplay(4096, (84, 84), 4, device=dev, seed=5, prioritized=cfg.prioritized_replay)
    rep.fill_synthetic(4096, 6, seed=5)
    ln = Learner(net, rep, cfg, use_graph=True)
    for _ in range(6):
        ln.step()
    torch.cuda.synchronize()
    return net, net.online.flat.clone()


for fuse in (0, 2):
    n0, a = run(fuse)
    _, b = run(fuse)
    lay = n0.layout
    diffs = {name: float((a[lay.offsets[name]:lay.offsets[name] + lay.numel(name)] -
                          b[lay.offsets[name]:lay.offsets[name] + lay.numel(name)]).abs().max()) for name in lay.names}
    print('fuse=%d run-to-run: bit-equal %s; nonzero max|diff|: %s' % (
        fuse, torch.equal(a, b), {k: '%.2e' % v for k, v in diffs.items() if v > 0}))
