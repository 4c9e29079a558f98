"""Device-op dispatch: HIP kernels for GPU tensors, PyTorch for CPU tensors.

Every function here has exactly one GPU implementation (the in-tree HIP
extension, `csrc/kernels/*.hip`) and one CPU implementation (plain torch,
which doubles as the numerics oracle in tests). GPU tensors never fall back
to torch silently: a missing extension raises (see `_ext.load(required=True)`).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from . import _ext


def _hip(t: torch.Tensor):
    if t.is_cuda:
        return _ext.load(required=True)
    return None


# ------------------------------------------------------------------ RNG (CPU)
def _cpu_gen(rng_state: torch.Tensor) -> torch.Generator:
    seed, ctr = int(rng_state[0]), int(rng_state[1])
    rng_state[1] += 1
    return torch.Generator().manual_seed((seed * 0x9E3779B1 + ctr * 0x85EBCA77) % (2 ** 63))


# --------------------------------------------------------------- replay ops
def replay_sample_uniform(size_dev: torch.Tensor, rng_state: torch.Tensor, out: torch.Tensor,
                          sample_out: Optional[list] = None):
    """out[i] = distinct uniform indices in [0, size) (without replacement).

    ``sample_out`` (GPU): [state_idx, next_idx, actions, rewards, dones, gammas,
    a_out, r_out, d_out, g_out, st_slots, nx_slots] gathers the per-sample
    scalars and the frame-slot tables of s / s' in the same launch."""
    ext = _hip(out)
    if ext is not None:
        ext.replay_sample_uniform(size_dev, rng_state, out, sample_out or [])
        return out
    n = int(size_dev[0])
    g = _cpu_gen(rng_state)
    B = out.numel()
    if n >= B:
        out.copy_(torch.randperm(n, generator=g)[:B].to(torch.int32))
    else:
        out.copy_(torch.randint(0, max(n, 1), (B,), generator=g).to(torch.int32))
    return out


def replay_gather_frames(frames: torch.Tensor, state_idx: torch.Tensor, next_idx: torch.Tensor,
                         idx: torch.Tensor, out: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
                         scalars: Optional[list] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Rebuild uint8 NHWC stacks: states [B,H,W,k], next_states [B,H,W,k].

    ``scalars`` = [actions, rewards, dones, gammas, a_out, r_out, d_out, g_out]
    gathers the per-sample columns in the same launch (GPU path)."""
    ext = _hip(frames)
    B, k = idx.numel(), state_idx.shape[1]
    H, W = frames.shape[1], frames.shape[2]
    if ext is not None:
        if out is None:
            s = torch.empty(B, H, W, k, dtype=torch.uint8, device=frames.device)
            ns = torch.empty_like(s)
        else:
            s, ns = out
        ext.replay_gather_frames(frames, state_idx, next_idx, idx, s, ns, scalars or [])
        return s, ns
    if scalars:
        for src, dst in zip(scalars[:4], scalars[4:]):
            dst.copy_(src.index_select(0, idx.long()))
    si = state_idx.index_select(0, idx.long()).long()                       # [B, k]
    ni = torch.cat([si[:, 1:], next_idx.index_select(0, idx.long()).long().view(B, 1)], 1)
    s = frames.index_select(0, si.reshape(-1)).view(B, k, H, W).permute(0, 2, 3, 1).contiguous()
    ns = frames.index_select(0, ni.reshape(-1)).view(B, k, H, W).permute(0, 2, 3, 1).contiguous()
    return s, ns


# -------------------------------------------------------------- sum-tree ops
def sumtree_set(tree, idx: torch.Tensor, td_abs: Optional[torch.Tensor], alpha: float, eps: float,
                use_max: bool):
    ext = _hip(tree.sum)
    if ext is not None:
        ext.sumtree_set(tree.sum, tree.min, tree.max_p, idx,
                        td_abs if td_abs is not None else tree.max_p, float(alpha), float(eps),
                        bool(use_max), tree.P)
        return
    P = tree.P
    leaf = idx.long() + P
    if use_max:
        p = tree.max_p.expand(leaf.numel()).clone()
    else:
        p = (td_abs.float() + eps) ** alpha
        tree.max_p.copy_(torch.maximum(tree.max_p, p.max().view(1)))
    # last writer wins for duplicate indices (sequential semantics)
    tree.sum[leaf] = p
    tree.min[leaf] = p
    nodes = leaf
    for _ in range(P.bit_length() - 1):          # log2(P) levels up to the root
        nodes = torch.unique(nodes // 2)
        tree.sum[nodes] = tree.sum[2 * nodes] + tree.sum[2 * nodes + 1]
        tree.min[nodes] = torch.minimum(tree.min[2 * nodes], tree.min[2 * nodes + 1])


def sumtree_sample(tree, rng_state, size_dev, beta, idx_out, w_out, sample_out: Optional[list] = None):
    """Stratified proportional sample + importance weights (max-normalised).

    beta: the IS exponent as a float tensor [1], or a ``(global_step, beta0, steps)`` schedule
    (int64 device step): the kernel anneals beta = min(1, beta0 + (1 - beta0) step / steps)
    itself, so a graph-captured learner step needs no host math or extra launches for it."""
    ext = _hip(tree.sum)
    sched = isinstance(beta, tuple)
    if ext is not None:
        if sched:
            step, b0, steps = beta
            ext.sumtree_sample(tree.sum, tree.min, rng_state, size_dev, step, idx_out, w_out, tree.P,
                               sample_out or [], float(b0), float(max(1, steps)))
        else:
            ext.sumtree_sample(tree.sum, tree.min, rng_state, size_dev, beta, idx_out, w_out, tree.P,
                               sample_out or [], 0.0, 1.0)
        return
    if sched:
        step, b0, steps = beta
        beta = torch.clamp(b0 + (1.0 - b0) * step.float() / max(1, steps), max=1.0)
    B, P = idx_out.numel(), tree.P
    g = _cpu_gen(rng_state)
    total = tree.sum[1]
    u = (torch.arange(B, dtype=torch.float32) + torch.rand(B, generator=g)) * (total / B)
    node = torch.ones(B, dtype=torch.long)
    while int(node[0]) < P:
        left = 2 * node
        ls = tree.sum[left]
        go_right = (u >= ls) & (tree.sum[left + 1] > 0)
        u = torch.where(go_right, u - ls, u)
        node = torch.where(go_right, left + 1, left)
    leaf = (node - P).clamp(max=int(size_dev[0]) - 1)
    idx_out.copy_(leaf.to(torch.int32))
    n = size_dev[0].float()
    p = tree.sum[leaf + P] / total
    pmin = tree.min[1] / total
    b = beta.float()
    w_out.copy_((n * p).pow(-b) / (n * pmin).pow(-b))


# ------------------------------------------------------------- optimizer op
def optimizer_step(opt, param: torch.Tensor, grad: torch.Tensor, grad_scale: float = 1.0,
                   global_step: Optional[torch.Tensor] = None, target: Optional[torch.Tensor] = None,
                   target_freq: int = 1):
    ext = _ext.load(required=True)
    from ..optim import kernel_op
    hp = opt.hp
    s0 = opt.slots[0] if len(opt.slots) > 0 else param
    s1 = opt.slots[1] if len(opt.slots) > 1 else param
    if getattr(opt, 'ticket', None) is None or opt.ticket.device != param.device:
        opt.ticket = torch.zeros(17 * 32, dtype=torch.int32, device=param.device)
    ext.optimizer_step(kernel_op(opt), param, grad, s0, s1, opt.beta_powers, opt.ticket,
                       float(opt.lr), float(opt.reg_param), int(opt.layout.reg_end),
                       float(grad_scale), global_step if global_step is not None else opt.beta_powers,
                       global_step is not None, [float(hp['momentum']), float(hp['rho']),
                                           float(hp['rms_mom']), float(hp['rms_eps']),
                                           float(hp['b1']), float(hp['b2']), float(hp['adam_eps']),
                                           float(hp['ad_rho']), float(hp['ad_eps'])],
                       target, int(target_freq))


# ---------------------------------------------------------- target network
def target_update(dst: torch.Tensor, src: torch.Tensor, tau: float,
                  step: Optional[torch.Tensor] = None, freq: int = 1, extra: Optional[tuple] = None):
    """dst = tau*src + (1-tau)*dst, executed only when step % freq == 0 (device predicate).

    ``extra`` = (dst2, src2): a second buffer pair hard-copied in the same launch
    under the same predicate (the executor's packed bf16 weights)."""
    ext = _hip(dst)
    if ext is not None:
        ext.target_update(dst, src, float(tau), step if step is not None else src, int(freq),
                          step is not None, list(extra) if extra else [])
        return
    if extra:
        target_update(extra[0], extra[1], 1.0, step, freq)
    if step is not None and int(step) % freq != 0:
        return
    if tau >= 1.0:
        dst.copy_(src)
    else:
        dst.mul_(1.0 - tau).add_(src, alpha=tau)
