"""Ape-X on the GPU (BASELINE config 4 shape, tiny): CPU actor processes, the native ingest
(csrc/host/apex_ingest.cpp) into the HBM PER replay, the native inference server thread
(csrc/infer_server.cpp) replaying captured inference graphs, and the multi-step learner graphs."""
import tempfile

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_apex_trainer_native_paths():
    from dist_dqn_amd.actors.apex import ApexActorPool, ApexTrainer
    from dist_dqn_amd.config import preset
    from dist_dqn_amd.learner import Learner
    from dist_dqn_amd.models.network import Network
    from dist_dqn_amd.replay import DeviceReplay
    dev = torch.device('cuda', 0)
    cfg = preset('apex', 'Pong-v0', '--num_actors=3 --replay_memory_capacity=20000 --replay_start_size=500 '
                 '--apex_ring=256 --logdir=%s' % tempfile.mkdtemp())
    net = Network.create_network(cfg, (84, 84, 4), 6, device=dev)
    rep = DeviceReplay(cfg.replay_memory_capacity, (84, 84), 4, device=dev, num_actors=cfg.num_actors,
                       prioritized=True, alpha=cfg.per_alpha, seed=1)
    ln = Learner(net, rep, cfg)
    pool = ApexActorPool(cfg.env, cfg.num_actors, 4, (84, 84), 0, 6, 200, seed=1, ring_capacity=cfg.apex_ring,
                         n_step=cfg.n_step, gamma=cfg.reward_discount)
    tr = ApexTrainer(net, rep, ln, pool, cfg)
    tr.run(max_seconds=12.0, log_every=100.0)
    assert getattr(tr, '_server', 'gone') is None, 'native server not stopped'
    assert pool.served > 0 and tr.serve_calls > 0, 'no greedy action served'
    assert pool.frames > 500 and rep.size() > 500
    assert ln.train_steps > 100 and ln.train_steps % cfg.apex_graph_steps == 0
    assert torch.isfinite(net.online.flat).all() and torch.isfinite(ln.loss).all()
