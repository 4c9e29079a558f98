"""Probe: phase stamps of the reference `cnn` net's fused per-sample kernels (csrc/kernels/cnn.hip)
in the production training step (s_memrealtime, 100 MHz), relative to each launch's first block:

  cnn_fwd  0 start  1 input staged  2 conv1  3 pool1  4 conv2  5 pool2  6 conv3  7 end
  cnn_bwd  0 start  1 loads  2 pool3  3 conv3 dgrad  4 pool2  5 conv2 dgrad  6 a1 staged  7 end

    python scripts/probe_cnn.py [--dtype=bf16|fp32] [extra config flags...]

Prints one JSON line: per phase, the [min, median, max] over blocks in us.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from dist_dqn_amd.actors.device_actor import DeviceActor
    from dist_dqn_amd.config import preset
    from dist_dqn_amd.learner import Learner
    from dist_dqn_amd.models.network import Network
    from dist_dqn_amd.replay import DeviceReplay
    dev = torch.device('cuda', 0)
    cfg = preset('atari', 'Pong-v0', '--seed=0 --dtype=bf16 --replay_memory_capacity=65536 ' + ' '.join(sys.argv[1:]))
    net = Network.create_network(cfg, (84, 84, 4), 6, device=dev)
    rep = DeviceReplay(65536, (84, 84), 4, device=dev)
    rep.fill_synthetic(65536, 6)
    actor = DeviceActor(net, rep, cfg, num_envs=4, steps_per_call=1, seed=3)
    learner = Learner(net, rep, cfg, use_graph=False, actor=actor if actor.can_fuse(cfg.minibatch_size) else None)
    ex = net.executor
    B = cfg.minibatch_size
    nb_f = B * 4
    ex.cnn_prof = (torch.zeros(nb_f * 8, dtype=torch.int64, device=dev), torch.zeros(B * 8, dtype=torch.int64, device=dev))
    out = {'dtype': ex.compute_dtype}
    for name, t, n in (('cnn_fwd', 0, nb_f), ('cnn_bwd', 1, B)):
        res = []
        for _ in range(5):
            ex.cnn_prof[t].zero_()
            learner.step()
            torch.cuda.synchronize()
            v = ex.cnn_prof[t].view(-1, 8).cpu()
            v = v[v[:, 0] > 0]
            t0 = int(v[:, 0].min())
            res.append([[round(float(x), 2) for x in torch.quantile((v[:, i] - t0).double() / 100.0,
                                                                    torch.tensor([0.0, 0.5, 1.0], dtype=torch.float64))]
                        for i in range(8)])
        out[name] = res[-1]
        out[name + '_blocks'] = int(v.shape[0])
    print(json.dumps(out))


if __name__ == '__main__':
    main()
