"""Fused MLP kernel (csrc/kernels/mlp.hip, the reference SimpleNetwork) vs the PyTorch
fp32 oracle executor: Q-values, TD loss, priorities and the full flat gradient, over
batch sizes that span one and several 128-sample chunks; then a learner step."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda', 0)


def _setup(extra='', B=100, A=2, D=4, seed=0, weighted=False):
    from dist_dqn_amd.config import parse_args
    from dist_dqn_amd.models.executor import TorchExecutor
    from dist_dqn_amd.models.network import Network
    cfg = parse_args(['--seed=%d' % seed, '--backend=hip', '--network=simple'] + extra.split())
    net = Network.create_network(cfg, (D,), A, device=DEV)
    assert type(net.executor).__name__ == 'HipMlpExecutor'
    g = torch.Generator(device=DEV).manual_seed(seed)
    net.online.flat.normal_(0.0, 0.4, generator=g)
    net.target.flat.normal_(0.0, 0.4, generator=g)
    oracle = TorchExecutor(net.arch, net.layout, input_scale=cfg.input_scale, loss=cfg.loss, oracle=True,
                           huber_delta=cfg.huber_delta, double_dqn=cfg.double_dqn)
    batch = {
        'states': torch.randn(B, D, device=DEV, generator=g),
        'next_states': torch.randn(B, D, device=DEV, generator=g),
        'actions': torch.randint(0, A, (B,), dtype=torch.int32, device=DEV, generator=g),
        'rewards': torch.randn(B, device=DEV, generator=g) * 2.0,
        'dones': (torch.rand(B, device=DEV, generator=g) < 0.2).float(),
        'gammas': torch.full((B,), 0.99, device=DEV),
    }
    if weighted:
        batch['weights'] = torch.rand(B, device=DEV, generator=g) + 0.5
    return net, oracle, batch


@pytest.mark.parametrize('B,A', [(1, 2), (100, 2), (300, 6)])
def test_mlp_q_values_match_oracle(B, A):
    net, oracle, batch = _setup(B=B, A=A)
    q = net.q_values(batch['states'])
    ref = oracle.q_values(net.online.flat, batch['states'])
    torch.testing.assert_close(q, ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize('extra', ['', '--double_dqn', '--loss=huber', '--double_dqn --loss=huber'])
@pytest.mark.parametrize('B,A,weighted', [(1, 2, False), (100, 2, False), (300, 6, True)])
def test_mlp_loss_and_grad_match_oracle(extra, B, A, weighted):
    net, oracle, batch = _setup(extra, B=B, A=A, weighted=weighted)
    g1 = torch.zeros_like(net.online.flat)
    l1, p1 = net.executor.loss_and_grad(net.online.flat, net.target.flat, batch, g1)
    g2 = torch.zeros_like(net.online.flat)
    l2, p2 = oracle.loss_and_grad(net.online.flat, net.target.flat, batch, g2)
    torch.testing.assert_close(l1.view(()), l2.view(()), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(p1, p2, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(g1, g2, rtol=1e-4, atol=1e-6)


def test_mlp_learner_graph_equals_eager():
    """CartPole-shaped learner on the GPU: HBM vector replay + fused MLP kernel + optimizer,
    HIP-graph replay == eager."""
    from dist_dqn_amd.config import parse_args
    from dist_dqn_amd.learner import Learner
    from dist_dqn_amd.models.network import Network
    from dist_dqn_amd.replay import DeviceReplay
    outs = []
    for graph in (False, True):
        cfg = parse_args(['--seed=1', '--backend=hip', '--network=simple', '--optimizer=adam', '--lr=0.001',
                          '--minibatch_size=100'])
        net = Network.create_network(cfg, (4,), 2, device=DEV)
        rep = DeviceReplay(4096, (4,), 1, device=DEV, seed=2)
        rep.fill_synthetic(4096, 2, seed=2)
        ln = Learner(net, rep, cfg, use_graph=graph)
        for _ in range(6):
            ln.step()
        torch.cuda.synchronize()
        assert torch.isfinite(ln.loss).all() and int(net.global_step) == 6
        outs.append(net.online.flat.clone())
    torch.testing.assert_close(outs[0], outs[1], rtol=1e-5, atol=1e-7)
