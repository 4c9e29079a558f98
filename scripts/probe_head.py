"""Phase timing (s_memtime) of the head kernel with fused acting: learner block 0 and the
fused acting block. Scalar head by default; pass e.g. `--distributional --noisy --dueling
--double_dqn --optimizer=adam` for the C51 training head."""
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
cfg = preset('nature', 'Pong-v0', '--dtype=bf16 --seed=0 --backend=hip --replay_memory_capacity=200000 ' + extra)
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
if net.arch.distributional:
    print('C51 learner block 0 wave 0 (cycles): loads + selection %.0f | target softmax %.0f | projection %.0f | '
          'CE + dlogits %.0f | block reduce %.0f | total %.0f'
          % (d(0, 1), d(1, 2), d(2, 3), d(3, 4), d(4, 5), d(0, 5)))
    if t[16]:
        print('C51 acting block, env 0 (cycles): prefetch + frames %.0f | Q row %.0f | decision + advance %.0f | total %.0f'
              % (d(16, 17), d(17, 18), d(18, 19), d(16, 19)))
else:
    print('learner block 0 (cycles): Q tile %.0f | TD loss + dQ %.0f | dH %.0f | total %.0f'
          % (d(0, 1), d(1, 2), d(2, 3), d(0, 3)))
    if t[16]:
        print('acting block, env 0 (cycles): frames + Q tile %.0f | barrier %.0f | decision + advance %.0f | total %.0f'
              % (d(16, 17), d(17, 18), d(18, 19), d(16, 19)))

