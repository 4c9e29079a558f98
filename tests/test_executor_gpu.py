"""Fused HIP executor (bf16 MFMA) vs the PyTorch fp32 oracle executor:
Q-values, TD loss, per-sample priorities and the full flat gradient."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda', 0)


def _setup(extra='', B=32, seed=0):
    from dist_dqn_amd.config import preset
    from dist_dqn_amd.models.executor import TorchExecutor
    from dist_dqn_amd.models.network import Network
    # 'cnn:' prefix = the reference network (SAME convs + max-pools, no input scaling)
    kind = 'atari' if extra.startswith('cnn:') else 'nature'
    extra = extra[4:] if extra.startswith('cnn:') else extra
    if '--dtype=' not in extra:           # (default: the bf16 production build; fp32 cases say so)
        extra += ' --dtype=bf16'
    cfg = preset(kind, 'Pong-v0', '--seed=%d --backend=hip %s' % (seed, extra))
    net = Network.create_network(cfg, (84, 84, 4), 6, device=DEV)
    assert net.executor.name == 'hip'
    want = 'fp16' if '--dtype=fp16' in extra else 'fp32' if '--dtype=fp32' in extra else 'bf16'
    assert net.executor.compute_dtype == want
    if want != 'bf16':
        assert net.executor.ext.__name__.endswith('_C_f16' if want == 'fp16' else '_C_f32')
    g = torch.Generator(device=DEV).manual_seed(seed)
    # larger-than-init weights so every layer carries signal
    net.online.flat.normal_(0.0, 0.03, generator=g)
    net.target.flat.normal_(0.0, 0.03, generator=g)
    net.executor.repack(net.online.flat)
    net.executor.repack(net.target.flat)
    net.reset_noise(generator=g)          # noisy nets: a fresh factorised noise sample
    oracle = TorchExecutor(net.arch, net.layout, input_scale=cfg.input_scale, loss=cfg.loss, oracle=True,
                           huber_delta=cfg.huber_delta, double_dqn=cfg.double_dqn)
    batch = {
        'states': torch.randint(0, 256, (B, 84, 84, 4), dtype=torch.uint8, device=DEV, generator=g),
        'next_states': torch.randint(0, 256, (B, 84, 84, 4), dtype=torch.uint8, device=DEV, generator=g),
        'actions': torch.randint(0, 6, (B,), dtype=torch.int32, device=DEV, generator=g),
        # rewards dominate the TD error so bf16 rounding of Q does not cancel it away
        'rewards': torch.randn(B, device=DEV, generator=g) * 5.0,
        'dones': (torch.rand(B, device=DEV, generator=g) < 0.2).float(),
        'gammas': torch.full((B,), 0.99, device=DEV),
    }
    return net, oracle, batch


def _rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


RAINBOW = '--distributional --noisy --dueling --double_dqn'


F16 = ' --dtype=fp16'
F32 = ' --dtype=fp32'


@pytest.mark.parametrize('extra', ['', '--dueling --double_dqn --loss=huber', '--distributional', '--noisy --dueling',
                                   RAINBOW, 'cnn:', 'cnn:--dueling', F16, RAINBOW + F16, 'cnn:' + F16,
                                   F32, RAINBOW + F32, 'cnn:' + F32])
def test_q_values_match_oracle(extra):
    net, oracle, batch = _setup(extra)
    q = net.q_values(batch['states'])
    q_ref = oracle.q_values(net.online.flat, batch['states'], net.noise)
    # fp32 build (the reference precision): only the summation order differs from the oracle
    assert _rel(q, q_ref) < (1e-4 if F32 in extra else 2e-2)


@pytest.mark.parametrize('extra,B,weighted', [('', 32, False), ('--dueling --double_dqn --loss=huber', 32, True),
                                             ('', 7, False), ('--double_dqn', 64, False),
                                             ('--distributional', 32, False), ('--noisy', 32, False),
                                             (RAINBOW, 32, True), (RAINBOW, 13, False),
                                             ('cnn:', 32, False), ('cnn:--dueling --double_dqn --loss=huber', 32, True),
                                             ('cnn:', 7, False), ('cnn:--double_dqn', 64, False),
                                             # fp16 MFMA build (_C_f16, static loss scale)
                                             (F16, 32, False), ('--dueling --double_dqn --loss=huber' + F16, 32, True),
                                             ('--double_dqn' + F16, 64, False), (RAINBOW + F16, 32, True),
                                             ('cnn:' + F16, 32, False),
                                             # fp32 build (_C_f32): the reference's precision
                                             (F32, 32, False), ('--dueling --double_dqn --loss=huber' + F32, 32, True),
                                             (RAINBOW + F32, 32, True), ('cnn:' + F32, 32, False)])
def test_loss_and_grad_match_oracle(extra, B, weighted):
    net, oracle, batch = _setup(extra, B)
    if weighted:
        gen = torch.Generator(device=DEV).manual_seed(11)
        batch['weights'] = torch.rand(B, device=DEV, generator=gen) + 0.5
    g_hip = torch.zeros_like(net.online.flat)
    g_ref = torch.zeros_like(net.online.flat)
    loss, prio = net.executor.loss_and_grad(net.online.flat, net.target.flat, batch, g_hip, net.noise,
                                            net.noise_target)
    loss_r, prio_r = oracle.loss_and_grad(net.online.flat, net.target.flat, batch, g_ref, net.noise,
                                          net.noise_target)
    torch.cuda.synchronize()
    if F32 in extra:
        # fp32 MFMA vs the fp32 oracle: summation order only (a ReLU input within rounding of
        # zero may still flip, so the gradient checks stay per-tensor)
        assert abs(float(loss) - float(loss_r)) / abs(float(loss_r)) < 1e-4
        assert _rel(prio, prio_r) < 1e-4
        assert _rel(g_hip, g_ref) < 1e-3
        for name in net.layout.names:
            o, n = net.layout.offsets[name], net.layout.numel(name)
            assert _rel(g_hip[o:o + n], g_ref[o:o + n]) < 2e-3, name
        return
    assert abs(float(loss) - float(loss_r)) / abs(float(loss_r)) < 3e-2
    assert _rel(prio, prio_r) < 3e-2
    # bf16 activations flip a few ReLU masks near zero; a flipped unit contributes its
    # whole gradient, so the relative L2 error scales like sqrt(flip fraction) (~5-9%)
    # while the direction and norm stay right: check cosine and norm ratio per tensor.
    for name in net.layout.names:
        o, n = net.layout.offsets[name], net.layout.numel(name)
        a, b = g_hip[o:o + n].float(), g_ref[o:o + n].float()
        cos = float(torch.nn.functional.cosine_similarity(a, b, dim=0))
        ratio = float(a.norm() / (b.norm() + 1e-12))
        # (reference cnn: unscaled 0..255 inputs make bf16 rounding of the activations
        # relatively larger, and Huber's clip region amplifies it: 5% norm tolerance)
        # (and the oracle's MIOpen conv algorithm choice moves its own rounding: cnn conv1's
        # cosine sits at 0.989-0.992 from run to run, hence 0.985 there)
        # (a bias gradient sums one row per sample: a single flipped unit of the unscaled cnn moves
        # its norm most, 5.9% seen once for the dueling value stream's fc bias under Huber)
        tol = (0.08 if n <= 1024 else 0.05) if extra.startswith('cnn:') else 0.03
        cmin = 0.985 if extra.startswith('cnn:') else 0.99
        assert cos > cmin and abs(ratio - 1.0) < tol, (name, cos, ratio)


@pytest.mark.parametrize('dtype,parts', [('bf16', 2), ('fp32', 2), ('bf16', 4), ('fp32', 4)])
def test_cnn_backward_two_parts_equals_one(dtype, parts):
    """Reference cnn backward with two workgroups per sample (KernelTuning cnn_bwd_parts=2, the
    default: the conv2 dgrad m-tiles and pool1 windows split) == one workgroup per sample: the same
    d(conv pre-activation) buffers bit for bit, the same gradient up to the wgrad atomics' order.
    Four parts also split each conv2 dgrad dot product in two K halves: equal up to rounding."""
    outs = []
    for np_ in (1, parts):
        net, _, batch = _setup('cnn:--dtype=%s --kernel_tuning=cnn_bwd_parts=%d' % (dtype, np_))
        assert net.executor.tuning.cnn_parts(dtype) == np_
        g = torch.zeros_like(net.online.flat)
        net.executor.loss_and_grad(net.online.flat, net.target.flat, batch, g, net.noise, net.noise_target)
        torch.cuda.synchronize()
        ws = net.executor._workspace(32, DEV)
        outs.append((g.clone(), [ws[k].clone() for k in ('dc1', 'dc2', 'dc3')]))
    for a, b in zip(outs[0][1], outs[1][1]):
        if parts == 2:
            assert torch.equal(a, b)
        else:                       # (four parts split each conv2 dgrad dot product in two halves)
            assert _rel(a, b) < (1e-5 if dtype == 'fp32' else 1e-2)
    torch.testing.assert_close(outs[0][0], outs[1][0], rtol=1e-3, atol=1e-6) if parts == 2 else \
        torch.testing.assert_close(outs[0][0], outs[1][0], rtol=1e-2, atol=1e-4)


@pytest.mark.parametrize('dtype', ['bf16', 'fp16'])
def test_learner_step_graph_equals_eager(dtype):
    """HIP-graph replay of the full SGD step == the same step run eagerly."""
    from dist_dqn_amd.config import preset
    from dist_dqn_amd.learner import Learner
    from dist_dqn_amd.models.network import Network
    from dist_dqn_amd.replay import DeviceReplay
    outs = []
    for graph in (False, True):
        cfg = preset('nature', 'Pong-v0', '--seed=3 --backend=hip --replay_memory_capacity=4096 --dtype=%s' % dtype)
        net = Network.create_network(cfg, (84, 84, 4), 6, device=DEV)
        rep = DeviceReplay(4096, (84, 84), 4, device=DEV, seed=5)
        rep.fill_synthetic(4096, 6, seed=5)
        ln = Learner(net, rep, cfg, use_graph=graph)
        for _ in range(6):
            ln.step()
        torch.cuda.synchronize()
        outs.append(net.online.flat.clone())
        assert int(net.global_step) == 6
    # wgrad combines M-chunks with fp32 atomics (order-dependent last bits)
    torch.testing.assert_close(outs[0], outs[1], rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize('extra', ['', '--double_dqn --dueling --prioritized_replay --n_step=3'])
def test_learner_step_many_equals_single_steps(extra):
    """Learner.step_many(k) (ONE graph holding k step bodies, the Ape-X learner loop) ==
    k separate step() replays."""
    from dist_dqn_amd.config import preset
    from dist_dqn_amd.learner import Learner
    from dist_dqn_amd.models.network import Network
    from dist_dqn_amd.replay import DeviceReplay
    outs = []
    for many in (False, True):
        cfg = preset('nature', 'Pong-v0', '--seed=3 --backend=hip --dtype=bf16 --replay_memory_capacity=4096 '
                     '--target_update_freq=5 ' + extra)
        net = Network.create_network(cfg, (84, 84, 4), 6, device=DEV)
        rep = DeviceReplay(4096, (84, 84), 4, device=DEV, seed=5, prioritized=cfg.prioritized_replay)
        rep.fill_synthetic(4096, 6, seed=5)
        ln = Learner(net, rep, cfg, use_graph=True)
        for _ in range(3):                     # eager warm-up + the single-step capture
            ln.step()
        if many:
            ln.step_many(4)
            ln.step_many(4)
        else:
            for _ in range(8):
                ln.step()
        torch.cuda.synchronize()
        assert int(net.global_step) == 11 and ln.train_steps == 11
        outs.append((net.online.flat.clone(), net.target.flat.clone()))
    # (conv weight gradients combine M-chunks with fp32 atomics: order-dependent last bits)
    torch.testing.assert_close(outs[0][0], outs[1][0], rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(outs[0][1], outs[1][1], rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize('slots', [False, True])
def test_fused_trunk_matches_layerwise(slots):
    """trunk.hip (conv1..conv3 in one launch, activations in LDS) == the three
    layer-wise implicit-GEMM launches, from NHWC stacks and from frame-ring slots."""
    net, _, batch = _setup('', 16)
    ex = net.executor
    B = 16
    g = torch.Generator(device=DEV).manual_seed(7)
    frames = torch.randint(0, 256, (40, 84, 84), dtype=torch.uint8, device=DEV, generator=g)
    sl = torch.randint(0, 40, (B, 4), dtype=torch.int32, device=DEV, generator=g)
    x = batch['states'] if not slots else sl
    fr = frames if slots else None
    p, f = ex.packed(net.online.flat), net.online.flat
    ws = ex._workspace(B, DEV)
    outs = []
    for fused in (False, True):
        ex.fused_trunk = fused
        for k in ('x1', 'x2', 'x3', 'h'):
            ws[k].zero_()
        ex._fwd_trunk([x, x], [p, p], [f, f], ws, B, 2, frames=fr)
        torch.cuda.synchronize()
        outs.append({k: ws[k][:2].clone() for k in ('x1', 'x2', 'x3', 'h')})
    ex.fused_trunk = True
    for k in ('x1', 'x2'):     # only the online instance keeps x1 / x2
        torch.testing.assert_close(outs[1][k][0].float(), outs[0][k][0].float(), rtol=2e-2, atol=2e-2)
    for k in ('x3', 'h'):
        for i in range(2):
            assert _rel(outs[1][k][i], outs[0][k][i]) < 1e-2, (k, i)
    if slots:    # the slot path sees the same pixels as a materialised NHWC stack
        st = frames[sl.long()].permute(0, 2, 3, 1).contiguous()
        ex._fwd_trunk([st], [p], [f], ws, B, 1)
        torch.cuda.synchronize()
        assert torch.equal(ws['x3'][0], outs[1]['x3'][0])


def test_fused_hard_target_sync():
    """Optimizer + repack carry the hard target copy (device predicate on global_step)."""
    from dist_dqn_amd.config import preset
    from dist_dqn_amd.learner import Learner
    from dist_dqn_amd.models.network import Network
    from dist_dqn_amd.replay import DeviceReplay
    cfg = preset('nature', 'Pong-v0', '--seed=3 --backend=hip --dtype=bf16 --replay_memory_capacity=4096 --target_update_freq=3')
    net = Network.create_network(cfg, (84, 84, 4), 6, device=DEV)
    rep = DeviceReplay(4096, (84, 84), 4, device=DEV, seed=5)
    rep.fill_synthetic(4096, 6, seed=5)
    ln = Learner(net, rep, cfg, use_graph=True)
    ex = net.executor
    for step in range(1, 8):
        ln.step()
        torch.cuda.synchronize()
        same = torch.equal(net.target.flat, net.online.flat)
        # bitwise (the packed buffer also holds fp32 bias copies: NaN patterns as bf16)
        same_p = torch.equal(ex.packed(net.target.flat).view(torch.int16), ex.packed(net.online.flat).view(torch.int16))
        assert same == same_p == (step % 3 == 0), step


def test_cnn_slot_batch_equals_materialised_batch():
    """Reference cnn: conv1 from frame-ring slots == from materialised NHWC stacks."""
    net, _, batch = _setup('cnn:--double_dqn', 16)
    g = torch.Generator(device=DEV).manual_seed(3)
    frames = torch.randint(0, 256, (64, 84, 84), dtype=torch.uint8, device=DEV, generator=g)
    s = torch.randint(0, 64, (16, 4), dtype=torch.int32, device=DEV, generator=g)
    ns = torch.randint(0, 64, (16, 4), dtype=torch.int32, device=DEV, generator=g)
    mat = dict(batch, states=frames[s.long()].permute(0, 2, 3, 1).contiguous(),
               next_states=frames[ns.long()].permute(0, 2, 3, 1).contiguous())
    slot = {k: v for k, v in batch.items() if k not in ('states', 'next_states')}
    slot.update(frames=frames, state_slots=s, next_slots=ns)
    outs = []
    for b in (mat, slot):
        gr = torch.zeros_like(net.online.flat)
        loss, prio = net.executor.loss_and_grad(net.online.flat, net.target.flat, b, gr)
        torch.cuda.synchronize()
        outs.append((loss.clone(), prio.clone(), gr))
    torch.testing.assert_close(outs[0][0], outs[1][0])
    torch.testing.assert_close(outs[0][1], outs[1][1])
    torch.testing.assert_close(outs[0][2], outs[1][2], rtol=1e-4, atol=1e-5)   # (fp32 atomics order)


def test_cnn_learner_graph_equals_eager():
    from dist_dqn_amd.config import preset
    from dist_dqn_amd.learner import Learner
    from dist_dqn_amd.models.network import Network
    from dist_dqn_amd.replay import DeviceReplay
    outs = []
    for graph in (False, True):
        cfg = preset('atari', 'Pong-v0', '--seed=3 --backend=hip --dtype=bf16 --replay_memory_capacity=4096')
        net = Network.create_network(cfg, (84, 84, 4), 6, device=DEV)
        assert net.executor.name == 'hip' and type(net.executor).__name__ == 'HipCnnExecutor'
        rep = DeviceReplay(4096, (84, 84), 4, device=DEV, seed=5)
        rep.fill_synthetic(4096, 6, seed=5)
        ln = Learner(net, rep, cfg, use_graph=graph)
        for _ in range(5):
            ln.step()
        torch.cuda.synchronize()
        outs.append(net.online.flat.clone())
    torch.testing.assert_close(outs[0], outs[1], rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize('network,extra', [('nature', ''), ('cnn', ''), ('nature', '--distributional --dueling'),
                                           ('nature', RAINBOW), ('nature', RAINBOW + ' --prioritized_replay')])
def test_fused_acting_matches_separate_actor(network, extra):
    """The device actors' step inside the learner launches (extra trunk/fc instance + one
    head workgroup) writes the same transitions / frames / eps as the stand-alone act_fused
    path with the same weights and RNG."""
    from dist_dqn_amd.actors.device_actor import DeviceActor
    from dist_dqn_amd.config import preset
    from dist_dqn_amd.learner import Learner
    from dist_dqn_amd.models.network import Network
    from dist_dqn_amd.replay import DeviceReplay
    outs = []
    for fused in (False, True):
        cfg = preset(network if network == 'nature' else 'atari', 'Pong-v0',
                     '--seed=4 --backend=hip --dtype=bf16 --replay_memory_capacity=65536 ' + extra)
        net = Network.create_network(cfg, (84, 84, 4), 6, device=DEV)
        rep = DeviceReplay(65536, (84, 84), 4, device=DEV, seed=5, prioritized=cfg.prioritized_replay)
        rep.fill_synthetic(65536, 6, seed=5)
        actor = DeviceActor(net, rep, cfg, num_envs=4, steps_per_call=1, seed=11, use_graph=False)
        assert actor.can_fuse(cfg.minibatch_size)
        ln = Learner(net, rep, cfg, use_graph=False, actor=actor if fused else None)
        assert (ln.actor is not None) == fused
        for _ in range(3):
            if not fused:
                actor.step()
            ln.step()
        torch.cuda.synchronize()
        cur = rep.cursor.clone()
        t0 = int(cur[0]) - 12
        outs.append(dict(cursor=cur, actions=rep.actions[t0:t0 + 12].clone(), rewards=rep.rewards[t0:t0 + 12].clone(),
                         eps=actor.eps.clone(), frames_done=actor.frames_done.clone(), stacks=actor.stacks.clone(),
                         frame=rep.frames[int(actor.stacks[0, -1])].clone()))
    a, b = outs
    for k in a:
        assert torch.equal(a[k], b[k]), k


@pytest.mark.parametrize('extra', ['--optimizer=rmsprop', '--optimizer=adam --dueling', 'cnn:--optimizer=momentum'])
def test_fused_update_and_pack_equals_optimizer_plus_repack(extra):
    """optim_pack_kernel (update + forward/dgrad fragments + fp32 bias copy in one launch)
    == the plain optimizer kernel followed by the pack kernel, bit for bit."""
    net, _, batch = _setup(extra + ' --reg_param=0.001')
    ex, opt = net.executor, net.optimizer
    g = torch.Generator(device=DEV).manual_seed(9)
    grad = torch.randn(net.online.flat.shape, device=DEV, generator=g) * 1e-2
    # the fused path updates only named tensors (the alignment padding between them
    # carries no gradient and no consumer): compare on the named regions
    lay = net.layout
    named = torch.zeros_like(grad, dtype=torch.bool)
    for n in lay.names:
        named[lay.offsets[n]:lay.offsets[n] + lay.numel(n)] = True
    grad[~named] = 0.0
    states = []
    for fused in (False, True):
        flat = net.online.flat.clone()
        slots = [s.clone() for s in opt.slots]
        bp = opt.beta_powers.clone()
        step = torch.zeros(1, dtype=torch.int64, device=DEV)
        o_slots, o_bp = opt.slots, opt.beta_powers
        opt.slots, opt.beta_powers = slots, bp
        try:
            for _ in range(2):
                if fused:
                    ex.update_and_pack(opt, flat, grad, 0.5, step)
                else:
                    opt.step(flat, grad, 0.5, step)
                    ex.repack(flat)
        finally:
            opt.slots, opt.beta_powers = o_slots, o_bp
        torch.cuda.synchronize()
        states.append((flat, [s.clone() for s in slots], bp, step, ex.packed(flat).clone()))
    (f0, s0, b0, st0, p0), (f1, s1, b1, st1, p1) = states
    assert torch.equal(f0, f1), float((f0 - f1).abs().max())
    assert torch.equal(b0, b1) and torch.equal(st0, st1)
    for a, b in zip(s0, s1):
        assert torch.equal(a[named], b[named]), float((a - b)[named].abs().max())
    assert torch.equal(p0.view(torch.int16), p1.view(torch.int16))


def _noisy_eff_ref(net, flat, noise):
    """Torch fp32 effective weights: mu + sigma * f(eps_in) f(eps_out) per noisy dense layer."""
    lay, eff = net.layout, flat.clone()
    f = lambda x: x.sign() * x.abs().sqrt()
    noff = 0
    for d in net.arch.dense_layers():
        if not d.noisy:
            continue
        ei, eo = f(noise[noff:noff + d.fin]), f(noise[noff + d.fin:noff + d.fin + d.fout])
        v = lambda n: flat[lay.offsets[n]:lay.offsets[n] + lay.numel(n)]
        ow, ob = lay.offsets[d.name + '/w'], lay.offsets[d.name + '/b']
        eff[ow:ow + d.fin * d.fout] = v(d.name + '/w') + (v(d.name + '/w_sigma').view(d.fin, d.fout)
                                                          * torch.outer(ei, eo)).view(-1)
        eff[ob:ob + d.fout] = v(d.name + '/b') + v(d.name + '/b_sigma') * eo
        noff += d.fin + d.fout
    return eff


@pytest.mark.parametrize('extra', [RAINBOW, '--noisy --dueling'])
def test_noisy_fused_update_mixes_next_noise(extra):
    """Noisy nets: apply_grads = ONE launch doing the optimizer step on mu AND sigma plus the
    mix + pack under the next online noise sample. The update equals the plain optimizer
    kernel bit for bit; the fp32 effective weights match torch; Q-values of the premixed
    online net match the fp32 oracle under the new noise."""
    net, oracle, batch = _setup(extra + ' --reg_param=0.001')
    ex, opt = net.executor, net.optimizer
    g = torch.Generator(device=DEV).manual_seed(9)
    grad = torch.randn(net.online.flat.shape, device=DEV, generator=g) * 1e-2
    lay = net.layout
    named = torch.zeros_like(grad, dtype=torch.bool)
    for n in lay.names:
        named[lay.offsets[n]:lay.offsets[n] + lay.numel(n)] = True
    grad[~named] = 0.0
    ref = net.online.flat.clone()
    slots = [s.clone() for s in opt.slots]
    bp, step = opt.beta_powers.clone(), net.global_step.clone()
    old_noise = net.noise.clone()
    # the fused kernel derives dL/dsigma = dL/dW_eff * f(e_in) f(e_out) under the current noise
    grad_ref = grad.clone()
    f = lambda x: x.sign() * x.abs().sqrt()
    sig, noff = torch.zeros_like(named), 0
    for d in net.arch.dense_layers():
        if not d.noisy:
            continue
        ei, eo = f(old_noise[noff:noff + d.fin]), f(old_noise[noff + d.fin:noff + d.fin + d.fout])
        for kind, fac in (('w', torch.outer(ei, eo).view(-1)), ('b', eo)):
            o, os_ = lay.offsets[d.name + '/' + kind], lay.offsets[d.name + '/' + kind + '_sigma']
            k = lay.numel(d.name + '/' + kind)
            grad_ref[os_:os_ + k] = grad[o:o + k] * fac
            sig[os_:os_ + k] = True
        noff += d.fin + d.fout
    net.grad.copy_(grad)
    assert net.apply_grads(0.5, target_freq=1000)
    o_slots, o_bp = opt.slots, opt.beta_powers
    opt.slots, opt.beta_powers = slots, bp
    try:
        opt.step(ref, grad_ref, 0.5, step)
    finally:
        opt.slots, opt.beta_powers = o_slots, o_bp
    torch.cuda.synchronize()
    assert not torch.equal(old_noise, net.noise), 'apply_grads draws the next online noise'
    mu = named & ~sig
    assert torch.equal(net.online.flat[mu], ref[mu]), float((net.online.flat - ref)[mu].abs().max())
    torch.testing.assert_close(net.online.flat[sig], ref[sig], rtol=1e-5, atol=1e-7)
    for a, b in zip(opt.slots, slots):
        assert torch.equal(a[mu], b[mu])
        torch.testing.assert_close(a[sig], b[sig], rtol=1e-4, atol=1e-9)
    eff = ex._eff[net.online.flat.data_ptr()]
    eff_ref = _noisy_eff_ref(net, ref, net.noise)
    fc = {lay.offsets[n + '/w'] for n in ('fcl', 'value/fcl', 'advantage/fcl') if n + '/w' in lay.offsets}
    for n in lay.names:
        o, k = lay.offsets[n], lay.numel(n)
        if o in fc or lay.kinds[n] in ('w_sigma', 'b_sigma'):
            continue                   # fc weights are consumed packed only; sigma has no eff
        torch.testing.assert_close(eff[o:o + k], eff_ref[o:o + k], rtol=1e-5, atol=1e-6, msg=n)
    q = net.q_values(batch['states'])
    q_ref = oracle.q_values(net.online.flat, batch['states'], net.noise)
    assert _rel(q, q_ref) < 2e-2


def test_rainbow_learner_keeps_online_premixed():
    """Graph-replayed Rainbow learner steps (target noise drawn per step, online noise drawn
    inside the fused optimizer): the online net's packed weights always reflect net.noise."""
    from dist_dqn_amd.config import preset
    from dist_dqn_amd.learner import Learner
    from dist_dqn_amd.models.executor import TorchExecutor
    from dist_dqn_amd.models.network import Network
    from dist_dqn_amd.replay import DeviceReplay
    cfg = preset('nature', 'Pong-v0', '--seed=3 --backend=hip --dtype=bf16 --replay_memory_capacity=4096 ' + RAINBOW)
    net = Network.create_network(cfg, (84, 84, 4), 6, device=DEV)
    rep = DeviceReplay(4096, (84, 84), 4, device=DEV, seed=5)
    rep.fill_synthetic(4096, 6, seed=5)
    ln = Learner(net, rep, cfg, use_graph=True)
    for _ in range(6):
        ln.step()
    torch.cuda.synchronize()
    assert int(net.global_step) == 6 and bool(torch.isfinite(net.online.flat).all())
    oracle = TorchExecutor(net.arch, net.layout, input_scale=cfg.input_scale, loss=cfg.loss, oracle=True,
                           huber_delta=cfg.huber_delta, double_dqn=cfg.double_dqn)
    x = torch.randint(0, 256, (16, 84, 84, 4), dtype=torch.uint8, device=DEV)
    assert _rel(net.q_values(x), oracle.q_values(net.online.flat, x, net.noise)) < 2e-2


@pytest.mark.parametrize('dtype', ['bf16', 'fp16'])
def test_rainbow_factorised_target_tracks_syncs(dtype, monkeypatch):
    """Rainbow's target keeps separate mu / sigma fc fragments (written only at a sync) and mixes
    its per-step noise in the fc forward (qnet.hip fc_fwd_fz_kernel): over graph-replayed steps
    that cross two fused hard syncs, its Q-values match the fp32 oracle on the target's master
    weights under the target noise after every step."""
    from dist_dqn_amd.config import preset
    from dist_dqn_amd.learner import Learner
    from dist_dqn_amd.models.executor import TorchExecutor
    from dist_dqn_amd.models.network import Network
    from dist_dqn_amd.replay import DeviceReplay
    cfg = preset('nature', 'Pong-v0', '--seed=4 --backend=hip --dtype=%s --replay_memory_capacity=4096 '
                 '--target_update_freq=3 --kernel_tuning=tfact=1 %s' % (dtype, RAINBOW))   # (opt-in)
    net = Network.create_network(cfg, (84, 84, 4), 6, device=DEV)
    ex = net.executor
    assert ex.tfact and net.target.flat.data_ptr() in ex._fact
    rep = DeviceReplay(4096, (84, 84), 4, device=DEV, seed=6)
    rep.fill_synthetic(4096, 6, seed=6)
    ln = Learner(net, rep, cfg, use_graph=True)
    oracle = TorchExecutor(net.arch, net.layout, input_scale=cfg.input_scale, loss=cfg.loss, oracle=True,
                           huber_delta=cfg.huber_delta, double_dqn=cfg.double_dqn)
    x = torch.randint(0, 256, (16, 84, 84, 4), dtype=torch.uint8, device=DEV)
    t0 = net.target.flat.clone()
    for i in range(7):
        ln.step()
        torch.cuda.synchronize()
        q = net.target_q_values(x)
        q_ref = oracle.q_values(net.target.flat, x, net.noise_target)
        assert _rel(q, q_ref) < 2e-2, (i, _rel(q, q_ref))
    assert int(net.global_step) == 7 and not torch.equal(t0, net.target.flat)
    # after the step-6 sync the target's master equals the online net as it was then; one more
    # update moved the online net on
    assert not torch.equal(net.online.flat, net.target.flat)


@pytest.mark.parametrize('extra,acting', [('', False), ('--double_dqn', False), ('', True)])
def test_fused_sampling_equals_sampler_launch(extra, acting):
    """Uniform minibatch drawn by an extra block of the previous step's optimizer launch
    (--fuse_sampling=2) or inside the trunk launch (1: every workgroup re-derives the batch,
    sample_dev.h) == the standalone sampler launch (0): same indices, same rng counter, same
    parameters after graph-replayed steps (with and without fused acting)."""
    from dist_dqn_amd.actors.device_actor import DeviceActor
    from dist_dqn_amd.config import preset
    from dist_dqn_amd.learner import Learner
    from dist_dqn_amd.models.network import Network
    from dist_dqn_amd.replay import DeviceReplay
    outs = []
    for fuse in (0, 1, 2):
        cfg = preset('nature', 'Pong-v0', '--seed=3 --backend=hip --dtype=bf16 --replay_memory_capacity=4096 '
                     '--fuse_sampling=%d %s' % (fuse, extra))
        net = Network.create_network(cfg, (84, 84, 4), 6, device=DEV)
        rep = DeviceReplay(4096, (84, 84), 4, device=DEV, seed=5)
        rep.fill_synthetic(4096, 6, seed=5)
        actor = DeviceActor(net, rep, cfg, num_envs=4, steps_per_call=1, seed=1000) if acting else None
        ln = Learner(net, rep, cfg, use_graph=True, actor=actor)
        assert (ln.actor is not None) == acting
        assert ln._sample_mode() == ('launch', 'trunk', 'opt')[fuse]
        for _ in range(6):
            ln.step()
        torch.cuda.synchronize()
        if fuse == 2:   # the batch of step 7 is already drawn: compare step 6's batch via a rerun
            assert ln._presampled
        outs.append((net.online.flat.clone(), rep.size_dev.clone()))
    (f0, s0), (f1, s1), (f2, s2) = outs
    assert torch.equal(s0, s1) and torch.equal(s0, s2)
    torch.testing.assert_close(f0, f1, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(f0, f2, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize('extra', ['--prioritized_replay --double_dqn --dueling',
                                   '--prioritized_replay ' + RAINBOW + ' --optimizer=adam'])
def test_per_fused_in_optimizer_equals_separate_launches(extra):
    """Prioritized replay with --fuse_sampling=2: the optimizer launch's extra block writes
    this step's priorities into the sum-tree (one wave) and draws the next prioritized batch
    == the separate sumtree_set / sumtree_sample launches (same tree, same IS weights, same
    parameters)."""
    from dist_dqn_amd.config import preset
    from dist_dqn_amd.learner import Learner
    from dist_dqn_amd.models.network import Network
    from dist_dqn_amd.replay import DeviceReplay
    outs = []
    for fuse in (0, 2):
        # (--det_wgrad: bit-reproducible conv weight gradients, so the two runs' priorities -- and
        #  with them the prioritized minibatches -- can only differ through the sampling paths)
        cfg = preset('nature', 'Pong-v0', '--seed=3 --backend=hip --dtype=bf16 --replay_memory_capacity=4096 '
                     '--det_wgrad=1 --fuse_sampling=%d %s' % (fuse, extra))
        net = Network.create_network(cfg, (84, 84, 4), 6, device=DEV)
        rep = DeviceReplay(4096, (84, 84), 4, device=DEV, seed=5, prioritized=True)
        rep.fill_synthetic(4096, 6, seed=5)
        ln = Learner(net, rep, cfg, use_graph=True)
        assert ln._sample_mode() == ('opt' if fuse == 2 else 'launch')
        for _ in range(6):
            ln.step()
        torch.cuda.synchronize()
        if fuse == 0:      # the fused run has already drawn step 7's batch: draw it here too
            rep.sample_slots(32, (net.global_step, cfg.per_beta0, cfg.per_beta_steps))
        else:
            assert ln._presampled
        torch.cuda.synchronize()
        b = rep.slot_batch(32)
        outs.append((net.online.flat.clone(), rep.tree.sum.clone(), rep.tree.min.clone(), rep.rng_state.clone(),
                     b['idx'].clone(), b['weights'].clone()))
    (f0, s0, m0, r0, i0, w0), (f1, s1, m1, r1, i1, w1) = outs
    assert torch.equal(r0, r1) and torch.equal(i0, i1)
    torch.testing.assert_close(s1, s0, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(m1, m0, rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(w1, w0, rtol=1e-4, atol=1e-6)
    if '--optimizer=adam' in extra:
        # the conv weight gradients sum M-chunk partials with fp32 atomics (arrival order sets
        # their last bits: scripts/probe_determinism.py shows two runs of ONE config differ the
        # same way), and Adam turns a gradient that cancels to ~0 into a ~lr * sign(g) step;
        # so per tensor the two runs' updates must agree in direction and size instead
        init = Network.create_network(cfg, (84, 84, 4), 6, device=DEV).online.flat
        lay = net.layout
        for name in lay.names:
            o, n = lay.offsets[name], lay.numel(name)
            d1, d0 = f1[o:o + n] - init[o:o + n], f0[o:o + n] - init[o:o + n]
            cos = float(torch.nn.functional.cosine_similarity(d1, d0, dim=0))
            ratio = float(d1.norm() / (d0.norm() + 1e-30))
            assert cos > 0.98 and abs(ratio - 1) < 0.03, (name, cos, ratio)
    else:
        torch.testing.assert_close(f1, f0, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize('extra', ['--prioritized_replay --double_dqn --dueling',
                                   '--prioritized_replay ' + RAINBOW + ' --optimizer=adam'])
def test_fused_acting_per_insert_in_optimizer(extra):
    """PER + fused acting: the actors' new transitions enter the sum-tree inside the optimizer
    launch's sampler block (one climb with this step's priorities, lanes ordered insert-first)
    == the acting launch inserting them itself: same tree, same next batch, same parameters."""
    from dist_dqn_amd.actors.device_actor import DeviceActor
    from dist_dqn_amd.config import preset
    from dist_dqn_amd.learner import Learner
    from dist_dqn_amd.models.network import Network
    from dist_dqn_amd.replay import DeviceReplay
    outs = []
    for defer in (False, True):
        # (--det_wgrad: bit-reproducible conv weight gradients: the runs' priorities can only
        #  differ through the insert paths)
        cfg = preset('nature', 'Pong-v0', '--seed=3 --backend=hip --dtype=bf16 --replay_memory_capacity=4096 '
                     '--det_wgrad=1 --fuse_sampling=2 ' + extra)
        net = Network.create_network(cfg, (84, 84, 4), 6, device=DEV)
        rep = DeviceReplay(4096, (84, 84), 4, device=DEV, seed=5, prioritized=True)
        rep.fill_synthetic(4096, 6, seed=5)
        actor = DeviceActor(net, rep, cfg, num_envs=4, steps_per_call=1, seed=1000)
        ln = Learner(net, rep, cfg, use_graph=True, actor=actor)
        ln.defer_per_insert = defer
        assert ln.actor is not None and ln._sample_mode() == 'opt' and ln._defer_per_insert() == defer
        for _ in range(6):
            ln.step()
        torch.cuda.synchronize()
        b = rep.slot_batch(32)
        outs.append((net.online.flat.clone(), rep.tree.sum.clone(), rep.tree.min.clone(), rep.tree.max_p.clone(),
                     b['idx'].clone(), b['weights'].clone(), rep.cursor.clone()))
    (f0, s0, m0, x0, i0, w0, c0), (f1, s1, m1, x1, i1, w1, c1) = outs
    assert torch.equal(c0, c1) and torch.equal(i0, i1)
    torch.testing.assert_close(x1, x0, rtol=1e-5, atol=0)     # (Adam: last bits, see below)
    torch.testing.assert_close(s1, s0, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(m1, m0, rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(w1, w0, rtol=1e-4, atol=1e-6)
    if '--optimizer=adam' not in extra:       # (Adam: see the test above -- atomics' arrival order)
        torch.testing.assert_close(f1, f0, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize('network,extra', [('nature', ''), ('nature', RAINBOW)])
def test_device_actor_inserts_max_priority(network, extra):
    """PER + device actors: each acting step's new transitions enter the sum-tree at the
    running max priority (one-wave insert inside the acting launch), and every ancestor
    stays the exact sum / min of its children."""
    from dist_dqn_amd.actors.device_actor import DeviceActor
    from dist_dqn_amd.config import preset
    from dist_dqn_amd.models.network import Network
    from dist_dqn_amd.replay import DeviceReplay
    cfg = preset(network, 'Pong-v0', '--seed=3 --backend=hip --dtype=bf16 --replay_memory_capacity=4096 --prioritized_replay '
                 + extra)
    net = Network.create_network(cfg, (84, 84, 4), 6, device=DEV)
    rep = DeviceReplay(4096, (84, 84), 4, device=DEV, seed=5, prioritized=True)
    rep.fill_synthetic(4096, 6, seed=5)
    g = torch.Generator(device=DEV).manual_seed(1)
    idx = torch.randint(0, 4096, (64,), dtype=torch.int32, device=DEV, generator=g)
    rep.update_priorities(idx, torch.rand(64, device=DEV, generator=g) * 5.0, 1e-6)   # raises max_p
    actor = DeviceActor(net, rep, cfg, num_envs=4, steps_per_call=1, seed=1000)
    for _ in range(3):
        t0 = int(rep.cursor[0])
        actor.step()
        torch.cuda.synchronize()
        P, mp = rep.tree.P, float(rep.tree.max_p)
        for e in range(4):
            leaf = (t0 + e) % 4096
            assert float(rep.tree.sum[P + leaf]) == mp and float(rep.tree.min[P + leaf]) == mp
    s, m = rep.tree.sum.cpu(), rep.tree.min.cpu()
    lvl = s[P:2 * P].clone()
    mn = m[P:2 * P].clone()
    while lvl.numel() > 1:
        lvl = lvl.view(-1, 2).sum(1)
        mn = mn.view(-1, 2).min(1).values
    torch.testing.assert_close(s[1], lvl[0], rtol=1e-5, atol=1e-3)
    assert float(m[1]) == float(mn[0])


@pytest.mark.parametrize('extra', ['', '--prioritized_replay ' + RAINBOW + ' --optimizer=adam'])
def test_step_many_with_fused_acting_equals_single_steps(extra):
    """k SGD steps replayed from ONE k-step graph (Learner.step_many, fused device acting riding
    in every step) == k one-step graph replays: same replay cursor / actor frames / global step,
    parameters equal up to the conv-gradient atomics' arrival order."""
    from dist_dqn_amd.actors.device_actor import DeviceActor
    from dist_dqn_amd.config import preset
    from dist_dqn_amd.learner import Learner
    from dist_dqn_amd.models.network import Network
    from dist_dqn_amd.replay import DeviceReplay
    outs = []
    for many in (False, True):
        cfg = preset('nature', 'Pong-v0', '--seed=3 --backend=hip --dtype=bf16 --replay_memory_capacity=4096 ' + extra)
        net = Network.create_network(cfg, (84, 84, 4), 6, device=DEV)
        rep = DeviceReplay(4096, (84, 84), 4, device=DEV, seed=5, prioritized='--prioritized_replay' in extra)
        rep.fill_synthetic(4096, 6, seed=5)
        actor = DeviceActor(net, rep, cfg, num_envs=4, steps_per_call=1, seed=1000)
        ln = Learner(net, rep, cfg, use_graph=True, actor=actor)
        assert ln.actor is not None
        init = net.online.flat.clone()
        for _ in range(4):
            ln.step()
        if many:
            ln.step_many(8)
            ln.step_many(8)
        else:
            for _ in range(16):
                ln.step()
        torch.cuda.synchronize()
        assert ln.train_steps == 20 and int(net.global_step) == 20
        outs.append((net.online.flat.clone(), rep.cursor.clone(), actor.env_frames))
    (f0, c0, e0), (f1, c1, e1) = outs
    assert torch.equal(c0, c1) and e0 == e1 == 20 * 4
    if '--optimizer=adam' in extra:     # (see test_per_fused_in_optimizer_equals_separate_launches)
        cos = float(torch.nn.functional.cosine_similarity(f1 - init, f0 - init, dim=0))
        ratio = float((f1 - init).norm() / ((f0 - init).norm() + 1e-30))
        assert cos > 0.98 and abs(ratio - 1) < 0.03, (cos, ratio)
    else:
        torch.testing.assert_close(f1, f0, rtol=1e-4, atol=1e-6)
