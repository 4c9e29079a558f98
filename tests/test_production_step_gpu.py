"""The production default SGD step against the PyTorch fp32 oracle, on EVERY tensor.

The step runs exactly as bench.py and the CLI run it: one HIP graph per step, the fc forward +
head fold (fc_head.hip), the fused weight-gradient + optimizer launch (conv weight gradients by
fp32 atomics, the fc gradient formed from the FcFuse rows), the next minibatch drawn by the
optimizer launch's sampler block, and (``acting``) the device actors' step fused into the
learner's launches. The minibatch, the target and (noisy nets) the noise sample a step consumes
are read BEFORE that step; the gradient the step applied is recovered from the update itself:

* RMSProp (TF, momentum 0; the reference's Atari optimizer): w' = w - lr g / sqrt(ms' + eps)
  with ms' read back, so g = (w - w') sqrt(ms' + eps) / lr exactly up to fp32 rounding;
* Adam (Rainbow): m' = b1 m + (1 - b1) g, so g = (m' - b1 m) / (1 - b1);

minus the decoupled L2 term reg * w on the regularised range, and compared per tensor with the
oracle's gradient on the same minibatch / weights / noise: cosine > 0.985 and norm within 5%.

Reference: the loss and the optimizer step, `/root/reference/src/network.py:141-157,198-202`.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda', 0)
VARIANTS = {
    'dqn': '',
    'dd': '--dueling --double_dqn --loss=huber',
    'rainbow': '--dueling --double_dqn --distributional --noisy --prioritized_replay --optimizer=adam',
    'ref': '',            # the reference's own `cnn` on its atari preset (/root/reference/src/network.py:317-424)
}
CAP = 65536            # large replay: the actors' 4 appends per step never touch the sampled rows


def _build(variant, acting, dtype='bf16'):
    from dist_dqn_amd.config import preset
    from dist_dqn_amd.learner import Learner
    from dist_dqn_amd.models.network import Network
    from dist_dqn_amd.replay import DeviceReplay
    lr = 0.0001 if variant == 'rainbow' else 0.01
    cfg = preset('atari' if variant == 'ref' else 'nature', 'Pong-v0',
                 '--seed=0 --backend=hip --dtype=%s --replay_memory_capacity=%d --lr=%g %s'
                 % (dtype, CAP, lr, VARIANTS[variant]))
    net = Network.create_network(cfg, (84, 84, 4), 6, device=DEV)
    g = torch.Generator(device=DEV).manual_seed(7)
    net.online.flat.normal_(0.0, 0.03, generator=g)      # every layer carries signal
    net.target.flat.normal_(0.0, 0.03, generator=g)
    net.refresh_packed()
    rep = DeviceReplay(CAP, (84, 84), 4, device=DEV, prioritized=cfg.prioritized_replay, seed=3)
    rep.fill_synthetic(CAP, 6, seed=3)
    actor = None
    if acting:
        from dist_dqn_amd.actors.device_actor import DeviceActor
        actor = DeviceActor(net, rep, cfg, num_envs=4, steps_per_call=1, seed=11)
        assert actor.can_fuse(cfg.minibatch_size)
    ln = Learner(net, rep, cfg, actor=actor)
    return cfg, net, rep, ln


@pytest.mark.parametrize('variant,acting,dtype', [('dqn', False, 'bf16'), ('dqn', True, 'bf16'), ('dd', True, 'bf16'),
                                                  ('rainbow', True, 'bf16'), ('ref', True, 'bf16'),
                                                  ('ref', True, 'fp32'), ('dqn', True, 'fp32')])
def test_production_step_matches_fp32_oracle_every_tensor(variant, acting, dtype):
    """(fp32: the reference's precision, held to the fp32 build's tolerances: cosine > 0.9999, norm
    within 0.2 %.)"""
    from dist_dqn_amd.models.executor import TorchExecutor
    cfg, net, rep, ln = _build(variant, acting, dtype)
    for _ in range(4):                         # eager warm-up, graph capture, then graph replays
        ln.step()
    torch.cuda.synchronize()
    assert ln._graphs is not None, 'the production step runs as a HIP graph'
    assert ln._sample_mode() == 'opt' and ln._presampled, 'next minibatch drawn by the optimizer launch'
    assert (ln.actor is not None) == acting
    ex = net.executor
    assert ex.can_fold_head(cfg.minibatch_size) or ex.dist, 'scalar heads run the fold'
    # ---- what the next step consumes: its minibatch (drawn by the last optimizer launch), weights,
    #      target, optimizer slots and (noisy) the noise samples mixed into the packed weights
    sb = rep.slot_batch(cfg.minibatch_size)
    idx = sb['idx'].clone()
    batch = {k: v.clone() for k, v in rep.gather(idx).items()}
    if 'weights' in sb:
        batch['weights'] = sb['weights'].clone()
    w0, tgt0 = net.online.flat.clone(), net.target.flat.clone()
    s0 = [s.clone() for s in net.optimizer.slots]
    noise = net.noise.clone() if getattr(net, 'noise', None) is not None else None
    tnoise = net.noise_target.clone() if getattr(net, 'noise_target', None) is not None else None
    ln.step()
    torch.cuda.synchronize()
    assert not torch.equal(net.online.flat, w0)
    opt = net.optimizer
    lay = net.layout
    reg = torch.zeros_like(w0)
    reg[:lay.reg_end] = float(cfg.reg_param)
    if cfg.optimizer == 'rmsprop':
        hp = opt.hp
        g_rec = (w0 - net.online.flat).double() * torch.sqrt(opt.slots[0].double() + float(hp['rms_eps'])) / float(opt.lr)
    else:
        assert cfg.optimizer == 'adam'
        b1 = float(opt.hp['b1'])
        g_rec = (opt.slots[0].double() - b1 * s0[0].double()) / (1.0 - b1)
    g_rec = (g_rec - reg.double() * w0.double()).float()
    oracle = TorchExecutor(net.arch, lay, input_scale=cfg.input_scale, loss=cfg.loss, oracle=True,
                           huber_delta=cfg.huber_delta, double_dqn=cfg.double_dqn)
    g_ref = torch.zeros_like(w0)
    oracle.loss_and_grad(w0, tgt0, batch, g_ref, noise, tnoise)
    torch.cuda.synchronize()
    checked = []
    for name in lay.names:
        o, k = lay.offsets[name], lay.numel(name)
        a, b = g_rec[o:o + k].double(), g_ref[o:o + k].double()
        if float(b.norm()) == 0.0:
            continue
        cos = float(torch.nn.functional.cosine_similarity(a, b, dim=0))
        ratio = float(a.norm() / b.norm())
        tol = (0.9999, 2e-3) if dtype == 'fp32' else (0.985, 0.05)
        assert cos > tol[0] and abs(ratio - 1.0) < tol[1], (variant, acting, dtype, name, cos, ratio)
        checked.append(name)
    # every tensor of the net (Nature: conv1..3, fcl, output / value + advantage streams; noisy: sigma too)
    assert len(checked) >= 10, checked
    assert any(n.startswith('conv1') for n in checked) and any('fcl' in n for n in checked)
