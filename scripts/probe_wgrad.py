"""Time the grouped weight-gradient launch of the flagship step by member subsets (conv1 /
conv2+conv3 / fc / output layer / all), replaying the captured member lists of a real step.
Prints microseconds per launch (HIP events over 200 launches)."""
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
cfg = preset('nature', 'Pong-v0', '--dtype=bf16 --seed=0 --backend=hip --replay_memory_capacity=200000 ' + extra)
net = Network.create_network(cfg, (84, 84, 4), 6, device=dev)
rep = DeviceReplay(200000, (84, 84), 4, device=dev, seed=0)
rep.fill_synthetic(200000, 6, seed=0)
ext = net.executor.ext
calls = []
orig = ext.qnet_wgrad_group


def spy(members, dims, scales):
    calls.append((members, dims, scales))
    return orig(members, dims, scales)


ext.qnet_wgrad_group = spy
ln = Learner(net, rep, cfg, use_graph=False)
for _ in range(3):
    ln.step()
torch.cuda.synchronize()
ext.qnet_wgrad_group = orig
members, dims, scales = calls[-1]
names = ['conv1', 'conv3', 'conv2', 'fc'] + ['head%d' % i for i in range(len(members) - 4)]
subsets = {'all': list(range(len(members))), 'conv1': [0], 'conv2+3': [1, 2], 'fc': [3],
           'head': list(range(4, len(members))), 'convs': [0, 1, 2], 'fc+head': list(range(3, len(members)))}
for name, idx in subsets.items():
    if not idx:
        continue
    m, d, s = [members[i] for i in idx], [dims[i] for i in idx], [scales[i] for i in idx]
    for _ in range(20):
        orig(m, d, s)
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    st.record()
    for _ in range(200):
        orig(m, d, s)
    en.record()
    torch.cuda.synchronize()
    print('wgrad %-8s %6.2f us' % (name, st.elapsed_time(en) * 1e3 / 200))
