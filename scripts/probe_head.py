"""Phase timing (s_memtime) of the scalar head kernel in the flagship configuration
(Nature-CNN, fused acting): learner block 0 and the fused acting block."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dist_dqn_amd.actors.device_actor import DeviceActor  # noqa: E402
from dist_dqn_amd.config import preset  # noqa: E402
from dist_dqn_amd.learner import Learner  # noqa: E402
from dist_dqn_amd.models.network import Network  # noqa: E402
from dist_dqn_amd.replay import DeviceReplay  # noqa: E402

extra = ' '.join(sys.argv[1:])
dev = torch.device('cuda', 0)
cfg = preset('nature', 'Pong-v0', '--seed=0 --backend=hip --replay_memory_capacity=200000 ' + extra)
net = Network.create_network(cfg, (84, 84, 4), 6, device=dev)
rep = DeviceReplay(200000, (84, 84), 4, device=dev, seed=0)
rep.fill_synthetic(200000, 6, seed=0)
actor = DeviceActor(net, rep, cfg, num_envs=4, steps_per_call=1, seed=1000)
ln = Learner(net, rep, cfg, actor=actor if actor.can_fuse(32) else None)
net.executor.head_prof = torch.zeros(32, dtype=torch.int64, device=dev)
for _ in range(30):
    if ln.actor is None:
        actor.step()
    ln.step()
torch.cuda.synchronize()
t = net.executor.head_prof.double().tolist()
d = lambda i, j: t[j] - t[i]
print('learner block 0 (cycles): Q tile %.0f | TD loss + dQ %.0f | dH %.0f | total %.0f'
      % (d(0, 1), d(1, 2), d(2, 3), d(0, 3)))
if t[16]:
    print('acting block (cycles): Q tile %.0f | decision + frames %.0f | advance %.0f | total %.0f'
          % (d(16, 17), d(17, 18), d(18, 19), d(16, 19)))

