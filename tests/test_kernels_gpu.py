"""HIP kernel numerics vs the PyTorch (CPU, fp32) oracle of the same op."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = 'cuda'


def _ext():
    from dist_dqn_amd.ops import _ext
    return _ext.load(required=True)


def test_extension_is_native():
    from dist_dqn_amd.ops import _ext
    assert _ext.available() and _ext.path().endswith('.so')


def test_sample_uniform_distinct_and_in_range():
    from dist_dqn_amd.ops import kernels
    for n, B in [(10000, 32), (100, 100), (5000, 512), (40, 64)]:
        size = torch.tensor([n], dtype=torch.int32, device=DEV)
        rng = torch.tensor([123, 0], dtype=torch.int64, device=DEV)
        out = torch.empty(B, dtype=torch.int32, device=DEV)
        seen = []
        for _ in range(20):
            kernels.replay_sample_uniform(size, rng, out)
            o = out.cpu().numpy()
            assert o.min() >= 0 and o.max() < n
            if n >= B:
                assert len(set(o.tolist())) == B       # without replacement (random.sample)
            seen.append(o)
        assert int(rng[1].item()) == 20                 # device-side counter advanced per call
        allv = np.concatenate(seen)
        if n >= 1000:
            assert abs(allv.mean() / n - 0.5) < 0.05


def test_gather_frames_matches_oracle():
    from dist_dqn_amd.ops import kernels
    F, H, W, K, C, B = 300, 84, 84, 4, 100, 32
    g = torch.Generator().manual_seed(0)
    frames = torch.randint(0, 256, (F, H, W), dtype=torch.uint8, generator=g)
    sidx = torch.randint(0, F, (C, K), dtype=torch.int32, generator=g)
    nidx = torch.randint(0, F, (C,), dtype=torch.int32, generator=g)
    idx = torch.randint(0, C, (B,), dtype=torch.int32, generator=g)
    s_ref, ns_ref = kernels.replay_gather_frames(frames, sidx, nidx, idx)
    s, ns = kernels.replay_gather_frames(frames.to(DEV), sidx.to(DEV), nidx.to(DEV), idx.to(DEV))
    assert torch.equal(s.cpu(), s_ref) and torch.equal(ns.cpu(), ns_ref)


def test_sumtree_set_and_sample():
    from dist_dqn_amd.replay.sumtree import DeviceSumTree
    from dist_dqn_amd.ops import kernels
    C = 1000
    t_cpu, t_gpu = DeviceSumTree(C, 'cpu'), DeviceSumTree(C, DEV)
    idx = torch.arange(C, dtype=torch.int32)
    t_cpu.set_max_priority(idx)
    t_gpu.set_max_priority(idx.to(DEV))
    g = torch.Generator().manual_seed(0)
    for _ in range(5):
        upd = torch.randint(0, C, (64,), dtype=torch.int32, generator=g)
        upd = torch.unique(upd).to(torch.int32)              # unique -> deterministic leaf values
        td = torch.rand(upd.numel(), generator=g) * 3
        t_cpu.update(upd, td, 0.6, 1e-6)
        t_gpu.update(upd.to(DEV), td.to(DEV), 0.6, 1e-6)
    torch.testing.assert_close(t_gpu.sum.cpu(), t_cpu.sum, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(t_gpu.min.cpu(), t_cpu.min, rtol=1e-6, atol=0)
    torch.testing.assert_close(t_gpu.max_p.cpu(), t_cpu.max_p)
    # sampling: proportional to priority
    rng = torch.tensor([7, 0], dtype=torch.int64, device=DEV)
    size = torch.tensor([C], dtype=torch.int32, device=DEV)
    beta = torch.tensor([0.4], device=DEV)
    counts = np.zeros(C)
    io = torch.empty(256, dtype=torch.int32, device=DEV)
    wo = torch.empty(256, device=DEV)
    for _ in range(200):
        t_gpu.sample(rng, size, beta, io, wo)
        np.add.at(counts, io.cpu().numpy(), 1)
        assert float(wo.max()) <= 1.0 + 1e-5 and float(wo.min()) > 0
    p = t_cpu.sum[t_cpu.P:t_cpu.P + C].numpy()
    expected = p / p.sum() * counts.sum()
    assert np.corrcoef(counts, expected)[0, 1] > 0.9


@pytest.mark.parametrize('B', [32, 64, 100])
def test_sumtree_update_duplicates_matches_cpu(B):
    """Batch updates with duplicate indices (B <= 64: the one-wave sorted climb; B > 64: the
    level-synchronous kernel) == the sequential CPU tree: last batch position wins a leaf,
    every ancestor exact, the min-tree and the running max too."""
    from dist_dqn_amd.replay.sumtree import DeviceSumTree
    C = 200_000                                     # 18 levels
    t_cpu, t_gpu = DeviceSumTree(C, 'cpu'), DeviceSumTree(C, DEV)
    t_cpu.set_max_priority(torch.arange(C, dtype=torch.int32))
    t_gpu.set_max_priority(torch.arange(C, dtype=torch.int32, device=DEV))
    g = torch.Generator().manual_seed(1)
    for it in range(8):
        upd = torch.randint(0, C, (B,), dtype=torch.int32, generator=g)
        upd[1::7] = upd[0]                          # duplicates, incl. adjacent leaves / shared paths
        upd[3] = (upd[2] ^ 1) if it % 2 else upd[3]
        td = torch.rand(B, generator=g) * 3
        if B > 64:                                  # concurrent duplicate writes: keep values equal
            td[1::7] = td[0]
        t_cpu.update(upd, td, 0.6, 1e-6)
        t_gpu.update(upd.to(DEV), td.to(DEV), 0.6, 1e-6)
    torch.testing.assert_close(t_gpu.sum.cpu(), t_cpu.sum, rtol=1e-6, atol=1e-6)
    # (leaf values are powf on the GPU vs torch.pow on the CPU: 1-ulp differences)
    torch.testing.assert_close(t_gpu.min.cpu(), t_cpu.min, rtol=1e-6, atol=0)
    torch.testing.assert_close(t_gpu.max_p.cpu(), t_cpu.max_p)


@pytest.mark.parametrize('name', ['sgd', 'momentum', 'rmsprop', 'adam', 'adagrad', 'adadelta', 'ftrl'])
def test_fused_optimizer_matches_oracle(name):
    from dist_dqn_amd.models import ParamStore, build_arch
    from dist_dqn_amd.optim import FlatOptimizer
    arch = build_arch('cnn', (84, 84, 4), 6)
    ps_c = ParamStore(arch).init_(0)
    ps_g = ParamStore(arch, DEV)
    ps_g.flat.copy_(ps_c.flat)
    o_c = FlatOptimizer(name, ps_c.layout, 'cpu', lr=0.01, reg_param=0.003)
    o_g = FlatOptimizer(name, ps_g.layout, DEV, lr=0.01, reg_param=0.003)
    step = torch.zeros(1, dtype=torch.int64, device=DEV)
    g = torch.Generator().manual_seed(1)
    for i in range(4):
        # (momentum-0 RMSProp stores its never-read `mom` slot only on requested steps: request
        # it for the last one, where the oracle's value is that step's update)
        o_g.request_slots(i == 3)
        gr = torch.randn(ps_c.layout.total, generator=g) * 0.1
        o_c.step(ps_c.flat, gr, 0.5)
        o_g.step(ps_g.flat, gr.to(DEV), 0.5, step)
    torch.testing.assert_close(ps_g.flat.cpu(), ps_c.flat, rtol=1e-5, atol=1e-6)
    for a, b in zip(o_g.slots, o_c.slots):
        torch.testing.assert_close(a.cpu(), b, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(o_g.beta_powers.cpu(), o_c.beta_powers if name == 'adam' else o_g.beta_powers.cpu())
    assert int(step.item()) == 4


def test_target_update_predicate_and_polyak():
    from dist_dqn_amd.ops import kernels
    src = torch.randn(4096, device=DEV)
    dst = torch.zeros(4096, device=DEV)
    step = torch.tensor([3], dtype=torch.int64, device=DEV)
    kernels.target_update(dst, src, 1.0, step, 2)
    assert float(dst.abs().sum()) == 0.0                  # 3 % 2 != 0 -> no copy
    step.fill_(4)
    kernels.target_update(dst, src, 1.0, step, 2)
    assert torch.equal(dst, src)
    d2 = torch.zeros(4096, device=DEV)
    kernels.target_update(d2, src, 0.1)
    torch.testing.assert_close(d2, 0.1 * src)


@pytest.mark.parametrize('kind,double,weighted', [('mse', False, False), ('huber', True, True)])
def test_td_loss_scalar_kernel(kind, double, weighted):
    from dist_dqn_amd.ops.td import td_loss
    B, A = 32, 6
    g = torch.Generator().manual_seed(2)
    q = torch.randn(B, A, generator=g) * 3
    qt, qo = torch.randn(B, A, generator=g), torch.randn(B, A, generator=g)
    a = torch.randint(0, A, (B,), generator=g, dtype=torch.int32)
    r = torch.randn(B, generator=g)
    d = (torch.rand(B, generator=g) < 0.2).float()
    gm = torch.full((B,), 0.99)
    w = torch.rand(B, generator=g) if weighted else None
    qc = q.clone().requires_grad_(True)
    lc, pc = td_loss(qc, a.long(), r, d, gm, qt, qo if double else None, w, kind)
    lc.backward()
    qg = q.to(DEV).requires_grad_(True)
    lg, pg = td_loss(qg, a.to(DEV), r.to(DEV), d.to(DEV), gm.to(DEV), qt.to(DEV), qo.to(DEV) if double else None,
                     w.to(DEV) if weighted else None, kind)
    lg.backward()
    torch.testing.assert_close(lg.cpu(), lc.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(pg.cpu(), pc, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(qg.grad.cpu(), qc.grad, rtol=1e-5, atol=1e-7)


def test_td_loss_c51_kernel():
    from dist_dqn_amd.ops.td import td_loss
    B, A, N = 16, 4, 51
    g = torch.Generator().manual_seed(3)
    lg = torch.randn(B, A, N, generator=g)
    lt, lo = torch.randn(B, A, N, generator=g), torch.randn(B, A, N, generator=g)
    a = torch.randint(0, A, (B,), generator=g, dtype=torch.int32)
    r = torch.randn(B, generator=g) * 3
    d = (torch.rand(B, generator=g) < 0.3).float()
    gm = torch.full((B,), 0.99)
    xc = lg.clone().requires_grad_(True)
    lc, pc = td_loss(xc, a.long(), r, d, gm, lt, lo, None, distributional=True)
    lc.backward()
    xg = lg.to(DEV).requires_grad_(True)
    lgpu, pg = td_loss(xg, a.to(DEV), r.to(DEV), d.to(DEV), gm.to(DEV), lt.to(DEV), lo.to(DEV), None,
                       distributional=True)
    lgpu.backward()
    torch.testing.assert_close(lgpu.cpu(), lc.detach(), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(pg.cpu(), pc, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(xg.grad.cpu(), xc.grad, rtol=1e-4, atol=1e-6)


def test_preprocess_batch_bit_exact():
    from dist_dqn_amd.ops.preprocess import preprocess_batch
    from dist_dqn_amd.utils.image import resize_image
    g = torch.Generator().manual_seed(4)
    fr = torch.randint(0, 256, (3, 210, 160, 3), dtype=torch.uint8, generator=g)
    out = preprocess_batch(fr.to(DEV), 84, 84).cpu().numpy()
    for i in range(3):
        np.testing.assert_array_equal(out[i], resize_image(fr[i].numpy(), 84, 84))


def test_device_actor_appends_consistent_transitions():
    from dist_dqn_amd.actors.device_actor import DeviceActor
    from dist_dqn_amd.config import preset
    from dist_dqn_amd.models.network import Network
    from dist_dqn_amd.replay import DeviceReplay
    cfg = preset('nature', 'Pong-v0', '--dtype=bf16 --seed=0 --replay_memory_capacity=1000')
    net = Network.create_network(cfg, (84, 84, 4), 6, device=torch.device(DEV))
    rep = DeviceReplay(1000, (84, 84), 4, device=DEV)
    actor = DeviceActor(net, rep, cfg, num_envs=8, steps_per_call=4, episode_len=5, use_graph=True)
    for _ in range(6):
        actor.step()
    torch.cuda.synchronize()
    assert rep.size() == 8 * 4 * 6 and actor.env_frames == 8 * 4 * 6
    assert actor.epsilon < 1.0
    # each non-terminal transition's next state is the following transition's state (same env)
    si = rep.state_idx[:rep.size()].cpu().numpy()
    ni = rep.next_idx[:rep.size()].cpu().numpy()
    dn = rep.dones[:rep.size()].cpu().numpy()
    E = 8
    for t in range(rep.size() - E):
        nxt = np.concatenate([si[t, 1:], [ni[t]]])
        if dn[t] == 0:
            np.testing.assert_array_equal(si[t + E], nxt)
        else:
            assert len(set(si[t + E].tolist())) == 1        # new episode: duplicated reset frame


@pytest.mark.parametrize('W', [2, 8])
def test_lowrank_dense_wgrad_matches_fp32(W):
    """The low-rank DP member (L_DENSE_WGRAD_LR): dW = X^T dH and db = sum dH over all W*32
    all-gathered rows, summed in 64-row chunks inside ONE block per weight tile (no atomics) ==
    the fp32 reference; db_zero stores zeros into the bias; two launches are bit-identical."""
    from dist_dqn_amd.ops import _ext
    ext = _ext.load(required=True)
    M, F, H = W * 32, 3136, 512
    g = torch.Generator(device=DEV).manual_seed(W)
    x = torch.rand(M, F, device=DEV, generator=g).to(torch.bfloat16)
    dh = (torch.randn(M, H, device=DEV, generator=g) * 0.1).to(torch.bfloat16)
    dw = torch.full((F, H), float('nan'), device=DEV)
    db = torch.full((H,), float('nan'), device=DEV)
    run = lambda zero: ext.qnet_wgrad(12, x.data_ptr(), [M, H, F, 0, 0, 0, 0, 0, 0, 0, 0], dh.data_ptr(), H,
                                      dw.data_ptr(), db.data_ptr(), 0, 0, H, H, 64, 64, 128, 1.0, False,
                                      mloop=(M + 63) // 64, db_zero=zero)
    run(False)
    torch.cuda.synchronize()
    ref_w = x.float().t() @ dh.float()
    ref_b = dh.float().sum(0)
    torch.testing.assert_close(dw, ref_w, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(db, ref_b, rtol=1e-4, atol=1e-4)
    w1 = dw.clone()
    run(True)
    torch.cuda.synchronize()
    assert torch.equal(dw, w1) and bool((db == 0).all())
