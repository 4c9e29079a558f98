"""The fc weight gradient formed inside the fused optimizer launch (optim.hip FcFuse) and the
production head kernels' loss / dL/dQ against a loss computed purely in torch.

* deferred fc gradient: a learner step whose optimizer launch forms dW_fc = X^T dH (and the fc
  bias gradient) from the rows, vs the same step with the gradient written by the grouped
  weight-gradient launch and read back (``--fuse_fc_wgrad=0``); every parameter, slot and
  packed fragment must agree (the fc bias to summation order);
* the same against the pure-torch fp32 oracle gradient of the fc layer;
* head_loss_kernel / c51_train_kernel: loss, dL/dQ (dL/dlogits) and dH of the kernel vs torch
  autograd of ``models/losses.py`` on the very hidden rows the kernel consumed (fp32 output
  layer in torch; the kernel's output layer runs on bf16 MFMA fragments);
* deterministic conv weight gradients (``--det_wgrad``: chunk-group partials summed by the
  optimizer launch in a fixed order): two identical runs are bit-identical, the result matches
  the fp32-atomics path to summation order and the fp32 oracle's conv gradients.

Reference: the optimizer site `/root/reference/src/network.py:198-202` (``minimize``) and the
loss `/root/reference/src/network.py:141-157`.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda', 0)
RAINBOW = '--distributional --noisy --dueling --double_dqn --optimizer=adam'


def _learner(extra, fuse, seed=0, B=32):
    from dist_dqn_amd.config import preset
    from dist_dqn_amd.learner import Learner
    from dist_dqn_amd.models.network import Network
    from dist_dqn_amd.replay import DeviceReplay
    kind = 'atari' if extra.startswith('cnn:') else 'nature'
    extra = extra[4:] if extra.startswith('cnn:') else extra
    cfg = preset(kind, 'Pong-v0', '--seed=%d --backend=hip --dtype=bf16 --minibatch_size=%d --fuse_fc_wgrad=%d '
                 '--replay_memory_capacity=4096 --reg_param=0.001 %s' % (seed, B, int(fuse), extra))
    net = Network.create_network(cfg, (84, 84, 4), 6, device=DEV)
    g = torch.Generator(device=DEV).manual_seed(seed + 1)
    # larger-than-init weights so every layer carries signal
    net.online.flat.normal_(0.0, 0.03, generator=g)
    net.target.flat.copy_(net.online.flat)
    net.refresh_packed()
    rep = DeviceReplay(4096, (84, 84), 4, device=DEV, seed=seed + 5, prioritized=cfg.prioritized_replay)
    rep.fill_synthetic(4096, 6)
    return net, Learner(net, rep, cfg, use_graph=False)


def _state(net):
    out = {'flat': net.online.flat.clone(), 'step': net.global_step.clone()}
    for i, s in enumerate(net.optimizer.slots):
        out['slot%d' % i] = s.clone()
    return out


@pytest.mark.parametrize('extra', ['', '--dueling --double_dqn --loss=huber', 'cnn:', RAINBOW,
                                   '--optimizer=rmsprop --prioritized_replay --double_dqn'])
def test_deferred_fc_grad_matches_materialised(extra):
    runs = []
    for fuse in (True, False):
        # (the conv / output-layer weight gradients in their own launch in both runs: the fused
        # weight-gradient launch is compared by test_split_update_matches_separate_wgrad)
        # (--det_wgrad: the conv weight gradients bit-reproducible, so every non-fc tensor must agree
        #  to the last bit; with fp32 atomics Adam's first step turned summation-order noise in a
        #  ~0 gradient into a +-lr step: a flaky comparison)
        net, learner = _learner(extra + ' --fuse_wgrad_update=0 --det_wgrad=1', fuse)
        assert learner._defer_fc == fuse
        learner.step()
        torch.cuda.synchronize()
        assert not net.executor.pending_fc()
        one = _state(net)
        for _ in range(2):
            learner.step()
        torch.cuda.synchronize()
        runs.append((net, one, _state(net)))
    (na, a1, a3), (_, b1, b3) = runs
    lay = na.layout
    fc = {n for n in lay.names if 'fcl/' in n}
    assert fc, lay.names
    for n in lay.names:
        o, k = lay.offsets[n], lay.numel(n)
        for key in a1:
            if key == 'step':
                continue
            x, y = a1[key][o:o + k], b1[key][o:o + k]
            if n not in fc:
                # after one step the other gradients come from the same launches (up to the conv
                # weight gradients' fp32 atomics: their summation order varies run to run)
                torch.testing.assert_close(x, y, rtol=1e-5, atol=1e-9, msg='%s %s' % (key, n))
            elif n.endswith('/w') or n.endswith('/w_sigma'):
                # dW: the same MFMA dot products over the same rows
                torch.testing.assert_close(x, y, rtol=1e-5, atol=1e-9, msg='%s %s' % (key, n))
            else:                      # the fc bias sums its rows in another order
                torch.testing.assert_close(x, y, rtol=1e-4, atol=1e-7, msg='%s %s' % (key, n))
            # two more steps carry that rounding downstream (Adam's normalised steps amplify it
            # elementwise: compare the tensors' relative L2 distance)
            u, w = a3[key][o:o + k].double(), b3[key][o:o + k].double()
            assert float((u - w).norm() / (w.norm() + 1e-30)) < 1e-3, ('3 steps', key, n)
    assert torch.equal(a3['step'], b3['step'])


@pytest.mark.parametrize('extra', ['', '--dueling --double_dqn --loss=huber', RAINBOW + ' --prioritized_replay',
                                   '--optimizer=adam --prioritized_replay'])
def test_split_update_matches_separate_wgrad(extra):
    """Split update (``--fuse_wgrad_update=1``): the conv / output-layer weight gradients run in
    the leading blocks of the optimizer's first launch beside the fc update, the other tensors
    in a second launch -- vs the grouped weight-gradient launch before one optimizer launch.
    Same math; the conv gradients' fp32 atomics sum 256-row chunk groups in another order."""
    runs = []
    for fw in (1, 0):
        net, learner = _learner(extra + ' --fuse_wgrad_update=%d' % fw, True)
        assert learner._defer_wgrad == bool(fw)
        learner.step()
        torch.cuda.synchronize()
        assert not net.executor.pending_fc()
        one = _state(net)
        for _ in range(2):
            learner.step()
        torch.cuda.synchronize()
        runs.append((net, one, _state(net)))
    (na, a1, a3), (_, b1, b3) = runs
    lay = na.layout
    for n in lay.names:
        o, k = lay.offsets[n], lay.numel(n)
        for key in a1:
            if key == 'step':
                continue
            x, y = a1[key][o:o + k], b1[key][o:o + k]
            torch.testing.assert_close(x, y, rtol=1e-4, atol=1e-7, msg=lambda m: '%s %s: %s' % (key, n, m))
            if 'prioritized' in extra:
                # (prioritized sampling turns the first step's rounding differences in |TD| into a
                # different next minibatch: only the first step is comparable)
                continue
            u, w = a3[key][o:o + k].double(), b3[key][o:o + k].double()
            assert float((u - w).norm() / (w.norm() + 1e-30)) < 1e-3, ('3 steps', key, n)
    assert torch.equal(a3['step'], b3['step'])
    assert int(a3['step']) == 3


def test_split_update_graph_many_matches_eager():
    """The split update captured as one-step and 8-step HIP graphs == eager steps (same
    minibatches: the optimizer's second launch draws the next one)."""
    states = []
    for graph in (False, True):
        net, learner = _learner('--fuse_wgrad_update=1', True, seed=3)
        learner.use_graph = graph
        for _ in range(3):                          # (graph: 2 eager warm-up steps, then a one-step graph)
            learner.step()
        if graph:
            assert learner.can_step_many()
            learner.step_many(8)
        else:
            for _ in range(8):
                learner.step()
        torch.cuda.synchronize()
        states.append(_state(net))
    a, b = states
    assert torch.equal(a['step'], b['step'])
    for key in a:
        if key != 'step':
            u, w = a[key].double(), b[key].double()
            assert float((u - w).norm() / (w.norm() + 1e-30)) < 1e-3, key


def test_rmsprop_mom_slot_written_only_when_requested():
    """Momentum-0 RMSProp: the `mom` slot (TF RMSProp_1, never read) is stored only on steps
    after request_slots(True) -- then it holds that step's update, w_before - w_after."""
    net, learner = _learner('--optimizer=rmsprop', True)
    opt = net.optimizer
    assert opt.defers_slots
    mom = opt.slots[1]
    learner.step()
    torch.cuda.synchronize()
    assert float(mom.abs().max()) == 0.0
    opt.request_slots(True)
    w0 = net.online.flat.clone()
    learner.step()
    torch.cuda.synchronize()
    upd = w0 - net.online.flat
    lay = net.layout
    for n in lay.names:
        o, k = lay.offsets[n], lay.numel(n)
        # (w_before - w_after rounds to the weights' ulp, ~2e-9 at |w| ~ 0.03)
        torch.testing.assert_close(mom[o:o + k], upd[o:o + k], rtol=1e-3, atol=2e-8, msg=n)
    assert float(mom.abs().max()) > 0.0
    opt.request_slots(False)
    before = mom.clone()
    learner.step()
    torch.cuda.synchronize()
    assert torch.equal(before, mom)


@pytest.mark.parametrize('extra', ['', '--dueling', 'cnn:'])
def test_deferred_fc_update_matches_fp32_oracle(extra):
    """One step's fc update (SGD, so w' = w - lr * g exactly) from the fused launch vs the
    PyTorch fp32 oracle's fc gradient on the same minibatch."""
    from dist_dqn_amd.models.executor import TorchExecutor
    net, learner = _learner(extra + ' --optimizer=sgd --lr=0.5 --fuse_sampling=0', True)
    cfg = net.config
    oracle = TorchExecutor(net.arch, net.layout, input_scale=cfg.input_scale, loss=cfg.loss, oracle=True,
                           huber_delta=cfg.huber_delta, double_dqn=cfg.double_dqn)
    w0 = net.online.flat.clone()
    tgt = net.target.flat.clone()
    learner.step()
    torch.cuda.synchronize()
    # the minibatch the step used: the learner's sampled indices, gathered as materialised states
    batch = learner.replay.gather(learner.idx)
    g_ref = torch.zeros_like(w0)
    oracle.loss_and_grad(w0, tgt, batch, g_ref, None, None)
    lay = net.layout
    for n in lay.names:
        if 'fcl/' not in n:
            continue
        o, k = lay.offsets[n], lay.numel(n)
        g = (w0[o:o + k] - net.online.flat[o:o + k]) / 0.5
        if n.endswith('/w'):
            g = g - 0.001 * w0[o:o + k]           # decoupled L2 on the fc weights (reg_param)
        ref = g_ref[o:o + k]
        cos = float(torch.nn.functional.cosine_similarity(g, ref, dim=0))
        ratio = float(g.norm() / (ref.norm() + 1e-12))
        assert cos > 0.985 and abs(ratio - 1.0) < 0.05, (n, cos, ratio)


def _head_torch(net, ws, B, batch, dist):
    """Pure-torch loss on the kernel's own hidden rows: (loss, dL/dout, dH). Dueling (scalar):
    dout = dL/dQ, dH = dL/dh through Q = V + A - mean(A) by autograd."""
    from dist_dqn_amd.models import losses
    ex, lay = net.executor, net.layout
    HH, A = ex.HH, ex.A
    hs = [ws['h'][i][:B * HH].view(B, HH).float() for i in range(3 if ex.double else 2)]
    flats = [net.online.flat, net.target.flat, net.online.flat]
    T = lambda f, n, *shape: f[lay.offsets[n]:lay.offsets[n] + lay.numel(n)].view(*shape)
    if ex.dueling and not dist:
        H = ex.HID

        def q_of(h, f):
            v = h[:, :H] @ T(f, 'value/output/w', H, 1) + T(f, 'value/output/b', 1)
            a = h[:, H:] @ T(f, 'advantage/output/w', H, A) + T(f, 'advantage/output/b', A)
            return v + a - a.mean(1, keepdim=True)
        h0 = hs[0].detach().requires_grad_(True)
        o0 = q_of(h0, flats[0])
        o0.retain_grad()
        outs = [None] + [q_of(h, f) for h, f in zip(hs[1:], flats[1:])]
        loss, _ = losses.scalar_td_loss(o0, batch['actions'], batch['rewards'], batch['dones'], outs[1].detach(),
                                        outs[2].detach() if ex.double else None, batch['gammas'],
                                        net.config.loss, net.config.huber_delta)
        loss.backward()
        # the kernels hand the advantage stream's dL/dA = dQ - mean(dQ) to the output layer
        dq = o0.grad
        return float(loss), dq - dq.mean(1, keepdim=True), h0.grad * (hs[0] > 0).float()
    W = lambda f: f[lay.offsets['output/w']:lay.offsets['output/w'] + lay.numel('output/w')].view(HH, -1)
    bias = lambda f: f[lay.offsets['output/b']:lay.offsets['output/b'] + lay.numel('output/b')]
    outs = [h @ W(f) + bias(f) for h, f in zip(hs, flats)]
    o0 = outs[0].detach().requires_grad_(True)
    if dist:
        N = ex.atoms
        v = net.arch
        loss, _ = losses.c51_loss(o0.view(B, A, N), batch['actions'], batch['rewards'], batch['dones'],
                                  outs[1].view(B, A, N), outs[2].view(B, A, N) if ex.double else None,
                                  batch['gammas'].view(-1, 1), v.v_min, v.v_max)
    else:
        loss, _ = losses.scalar_td_loss(o0, batch['actions'], batch['rewards'], batch['dones'], outs[1],
                                        outs[2] if ex.double else None, batch['gammas'],
                                        net.config.loss, net.config.huber_delta)
    loss.backward()
    dout = o0.grad
    dh = (dout @ W(net.online.flat).t()) * (hs[0] > 0).float()
    return float(loss), dout, dh


@pytest.mark.parametrize('extra,fold', [('', True), ('', False), ('--double_dqn --loss=huber', True),
                                        ('--double_dqn --loss=huber', False), ('--dueling --double_dqn', True),
                                        ('--dueling', False), ('--distributional', False),
                                        ('--distributional --double_dqn', False)])
def test_head_kernels_match_pure_torch_loss(extra, fold):
    """The scalar head folded into the fc launch (fc_head.hip, fold) / head_loss_kernel /
    c51_train_kernel vs torch autograd on the same hidden rows: the loss, the dL/dQ
    (dL/dlogits) rows the kernel hands to the output layer's weight gradient, and dH."""
    from dist_dqn_amd.config import preset
    from dist_dqn_amd.models.network import Network
    B = 32
    cfg = preset('nature', 'Pong-v0', '--seed=3 --backend=hip --dtype=bf16 %s' % extra)
    net = Network.create_network(cfg, (84, 84, 4), 6, device=DEV)
    g = torch.Generator(device=DEV).manual_seed(4)
    net.online.flat.normal_(0.0, 0.03, generator=g)
    net.target.flat.normal_(0.0, 0.03, generator=g)
    net.refresh_packed()
    batch = {
        'states': torch.randint(0, 256, (B, 84, 84, 4), dtype=torch.uint8, device=DEV, generator=g),
        'next_states': torch.randint(0, 256, (B, 84, 84, 4), dtype=torch.uint8, device=DEV, generator=g),
        'actions': torch.randint(0, 6, (B,), dtype=torch.int32, device=DEV, generator=g),
        'rewards': torch.randn(B, device=DEV, generator=g) * 5.0,
        'dones': (torch.rand(B, device=DEV, generator=g) < 0.2).float(),
        'gammas': torch.full((B,), 0.99, device=DEV),
    }
    ex = net.executor
    ex.fold_head = fold
    assert ex.can_fold_head(B) == (fold and not ex.dist)
    grad = torch.zeros_like(net.online.flat)
    loss, _ = ex.loss_and_grad(net.online.flat, net.target.flat, batch, grad, None, None)
    torch.cuda.synchronize()
    ws = ex._workspace(B, DEV)
    dist = ex.dist
    loss_ref, dout_ref, dh_ref = _head_torch(net, ws, B, batch, dist)
    assert abs(float(loss) - loss_ref) / abs(loss_ref) < 1e-2, (float(loss), loss_ref)
    width = ex.c51_KD if dist else 64
    dq = ws['dq16'][:B * width].view(B, width)[:, :dout_ref.shape[1]].float()
    rel = lambda a, b: float((a - b).norm() / (b.norm() + 1e-12))
    assert rel(dq, dout_ref) < 2e-2, rel(dq, dout_ref)
    dh = ws['dh'][:B * ex.HH].view(B, ex.HH).float()
    assert rel(dh, dh_ref) < 3e-2, rel(dh, dh_ref)
    dh_bits, dq_bits = ws['dh'][:B * ex.HH].clone(), ws['dq16'][:B * width].clone()
    if fold:
        # the fold leaves its row-group counters zero: a second call is bit-identical
        fw = ex._fold_ws(B, DEV)
        assert not fw['cnt'].any()
        grad2 = torch.zeros_like(grad)
        loss2, _ = ex.loss_and_grad(net.online.flat, net.target.flat, batch, grad2, None, None)
        torch.cuda.synchronize()
        assert float(loss2) == float(loss)
        assert torch.equal(ws['dh'][:B * ex.HH], dh_bits) and torch.equal(ws['dq16'][:B * width], dq_bits)


def test_folded_head_dq_wait_timeout_raises(monkeypatch):
    """Spin-mode fold with the tails' dQ publish switched off (DQN_DEBUG_FOLD_NO_PUBLISH, read at
    launch): every waiting dH block gives up after 1 s, writes a zero dH tile and sets the fold's
    error word, and the learner's device check raises instead of training on stale dQ."""
    net, learner = _learner('', True)
    learner.step()                                   # a normal step: no error word
    torch.cuda.synchronize()
    learner._device_checks()
    assert net.executor.fold_errors() == []
    monkeypatch.setenv('DQN_DEBUG_FOLD_NO_PUBLISH', '1')
    learner.step()
    torch.cuda.synchronize()
    monkeypatch.delenv('DQN_DEBUG_FOLD_NO_PUBLISH')
    errs = net.executor.fold_errors()
    assert errs and all(e >> 24 == 1 for e in errs), errs
    # the waiting blocks wrote ZERO dH tiles (no stale previous-step rows): only the groups' tails
    # (one block per 16-row group) wrote their own tile
    dh = net.executor._workspace(learner.B, net.device)['dh'].float()
    assert float((dh == 0).float().mean()) > 0.9, float((dh == 0).float().mean())
    with pytest.raises(RuntimeError, match='folded head'):
        learner._device_checks()


@pytest.mark.parametrize('extra,B', [('', 32), ('--double_dqn --loss=huber', 32), ('--dueling --double_dqn', 32),
                                     ('cnn:--dueling', 32), ('--dueling', 256)])
def test_folded_head_gradient_matches_separate_head(extra, B):
    """One launch for fc + output layer + TD loss + dQ / dH (fc_head.hip) vs the fc igemm launch +
    head_loss_kernel on the same minibatch: the whole flat gradient, the loss and the priorities
    (the fold's output layer is fp32 on the stored bf16 h; the head kernel's bf16 MFMA fragments).
    B = 32: every block resident, the online blocks write their own dH tiles after the group's tail
    publishes dQ (spin mode); B = 256: more blocks than CUs, the tails write the whole dH."""
    from dist_dqn_amd.config import preset
    from dist_dqn_amd.models.network import Network
    kind = 'atari' if extra.startswith('cnn:') else 'nature'
    extra = extra[4:] if extra.startswith('cnn:') else extra
    outs = []
    for fold in (True, False):
        cfg = preset(kind, 'Pong-v0', '--seed=3 --backend=hip --dtype=bf16 --minibatch_size=%d %s' % (B, extra))
        net = Network.create_network(cfg, (84, 84, 4), 6, device=DEV)
        g = torch.Generator(device=DEV).manual_seed(4)
        net.online.flat.normal_(0.0, 0.03, generator=g)
        net.target.flat.normal_(0.0, 0.03, generator=g)
        net.refresh_packed()
        batch = {
            'states': torch.randint(0, 256, (B, 84, 84, 4), dtype=torch.uint8, device=DEV, generator=g),
            'next_states': torch.randint(0, 256, (B, 84, 84, 4), dtype=torch.uint8, device=DEV, generator=g),
            'actions': torch.randint(0, 6, (B,), dtype=torch.int32, device=DEV, generator=g),
            'rewards': torch.randn(B, device=DEV, generator=g) * 5.0,
            'dones': (torch.rand(B, device=DEV, generator=g) < 0.2).float(),
            'gammas': torch.full((B,), 0.99, device=DEV),
        }
        ex = net.executor
        ex.fold_head = fold
        grad = torch.zeros_like(net.online.flat)
        loss, prio = ex.loss_and_grad(net.online.flat, net.target.flat, batch, grad, None, None)
        torch.cuda.synchronize()
        outs.append((float(loss), prio.clone(), grad.clone(), net.layout))
    (la, pa, ga, lay), (lb, pb, gb, _) = outs
    assert abs(la - lb) / abs(lb) < 5e-3, (la, lb)
    # |TD| per sample: both heads round differently (bf16 output-layer fragments vs fp32), an
    # error on the scale of Q, not of each |TD|
    torch.testing.assert_close(pa, pb, rtol=0, atol=2e-2 * float(pb.abs().max()))
    for n in lay.names:
        o, k = lay.offsets[n], lay.numel(n)
        x, y = ga[o:o + k].double(), gb[o:o + k].double()
        assert float((x - y).norm() / (y.norm() + 1e-30)) < 2e-2, n


@pytest.mark.parametrize('extra', ['', RAINBOW])
def test_det_wgrad_bitwise_reproducible(extra):
    """Same seed, same minibatches: with the deterministic conv weight gradients every parameter
    and slot is bit-identical after several steps (the atomics path differs run to run in the
    last bits); against the atomics path the first step agrees to summation order."""
    states = []
    for det in (1, 1, 0):
        net, learner = _learner(extra + ' --det_wgrad=%d' % det, True)
        assert learner._det_wgrad == bool(det)
        learner.step()
        torch.cuda.synchronize()
        assert not net.executor.pending_fc()
        one = _state(net)
        for _ in range(3):
            learner.step()
        torch.cuda.synchronize()
        states.append((one, _state(net)))
    (a1, a4), (b1, b4), (c1, _) = states
    lr = float(net.optimizer.lr)
    for key in a4:
        assert torch.equal(a1[key], b1[key]) and torch.equal(a4[key], b4[key]), key
        # against the atomics path: summation order only. Adam's first step is ~lr * sign(g) where
        # a conv gradient cancels to ~eps, so a few such elements may move by up to ~lr; every
        # other element agrees to 1e-5
        d = (a1[key] - c1[key]).abs()
        bad = d > 1e-9 + 1e-5 * c1[key].abs()
        assert float(bad.float().mean()) < 1e-4 and float(d.max()) <= 2.5 * lr, \
            (key, int(bad.sum()), float(d.max()))


def test_det_wgrad_conv_update_matches_fp32_oracle():
    """One SGD step's conv weight / bias updates from the partial sums vs the PyTorch fp32
    oracle's gradient on the same minibatch."""
    from dist_dqn_amd.models.executor import TorchExecutor
    net, learner = _learner('--optimizer=sgd --lr=0.5 --fuse_sampling=0 --det_wgrad=1', True)
    assert learner._det_wgrad
    cfg = net.config
    oracle = TorchExecutor(net.arch, net.layout, input_scale=cfg.input_scale, loss=cfg.loss, oracle=True,
                           huber_delta=cfg.huber_delta, double_dqn=cfg.double_dqn)
    w0 = net.online.flat.clone()
    tgt = net.target.flat.clone()
    learner.step()
    torch.cuda.synchronize()
    batch = learner.replay.gather(learner.idx)
    g_ref = torch.zeros_like(w0)
    oracle.loss_and_grad(w0, tgt, batch, g_ref, None, None)
    lay = net.layout
    seen = 0
    for n in lay.names:
        if not n.startswith('conv'):
            continue
        o, k = lay.offsets[n], lay.numel(n)
        g = (w0[o:o + k] - net.online.flat[o:o + k]) / 0.5
        ref = g_ref[o:o + k]
        cos = float(torch.nn.functional.cosine_similarity(g, ref, dim=0))
        ratio = float(g.norm() / (ref.norm() + 1e-12))
        assert cos > 0.98 and abs(ratio - 1.0) < 0.05, (n, cos, ratio)
        seen += 1
    assert seen == 6


@pytest.mark.parametrize('extra', ['', '--dueling --double_dqn --loss=huber', RAINBOW])
def test_dgrad_chain_matches_separate_launches(extra):
    """fc dgrad -> conv3 dgrad (-> conv2 dgrad) in ONE launch (dgrad_chain_kernel: stages wait on
    per-sample counters, producers store write-through) vs the three launches: the same dz3 / dz2 /
    dz1 bit for bit (same GEMMs, same split-K order) over two steps, and the same gradients."""
    from dist_dqn_amd.config import preset
    from dist_dqn_amd.models.network import Network
    B = 32
    outs = []
    for chain in (1, 2, 0):
        cfg = preset('nature', 'Pong-v0', '--seed=3 --backend=hip --dtype=bf16 %s' % extra)
        net = Network.create_network(cfg, (84, 84, 4), 6, device=DEV)
        g = torch.Generator(device=DEV).manual_seed(4)
        net.online.flat.normal_(0.0, 0.03, generator=g)
        net.target.flat.normal_(0.0, 0.03, generator=g)
        net.refresh_packed()
        ex = net.executor
        ex.chain_dgrad = chain                  # (opt-in: the default is 0, measured faster)
        assert bool(ex.can_chain_dgrad(B)) == bool(chain)
        res = []
        for it in range(2):
            batch = {
                'states': torch.randint(0, 256, (B, 84, 84, 4), dtype=torch.uint8, device=DEV, generator=g),
                'next_states': torch.randint(0, 256, (B, 84, 84, 4), dtype=torch.uint8, device=DEV, generator=g),
                'actions': torch.randint(0, 6, (B,), dtype=torch.int32, device=DEV, generator=g),
                'rewards': torch.randn(B, device=DEV, generator=g) * 5.0,
                'dones': (torch.rand(B, device=DEV, generator=g) < 0.2).float(),
                'gammas': torch.full((B,), 0.99, device=DEV),
            }
            grad = torch.zeros_like(net.online.flat)
            noise, tnoise = (net.noise, net.noise_target) if ex.noisy else (None, None)
            loss, _ = ex.loss_and_grad(net.online.flat, net.target.flat, batch, grad, noise, tnoise)
            torch.cuda.synchronize()
            ws = ex._workspace(B, DEV)
            res.append((ws['dz3'].clone(), ws['dz2'].clone(), ws['dz1'].clone(), float(loss), grad.clone()))
        if chain:
            assert not ex.chain_error(B, DEV)
        outs.append(res)
    for run in outs[:2]:                      # the 2-stage and the 3-stage chain vs separate launches
        for (a3, a2, a1, la, ga), (b3, b2, b1, lb, gb) in zip(run, outs[2]):
            assert torch.equal(a3, b3) and torch.equal(a2, b2) and torch.equal(a1, b1)
            assert la == lb
            torch.testing.assert_close(ga, gb, rtol=1e-4, atol=1e-7)
