"""TD losses (torch oracle; the fused HIP kernel is `csrc/kernels/td_loss.hip`).

Reference loss (`/root/reference/src/network.py:141-157`, targets built on
the host at `/root/reference/src/dqn_agent.py:224-253`):
    y  = r + gamma * max_a' Q_target(s', a')   (y = r when terminal)
    L  = mean((Q(s, a) - y)^2) + reg_param * sum_w 0.5 ||w||^2
Extensions: Huber, Double DQN (argmax by the online net), n-step discount
(gamma_n = gamma ** n), importance weights (PER), and the C51 categorical
projection loss. The L2 term is NOT part of these functions: it is applied
as ``grad += reg_param * w`` in the optimizer (same gradient, no extra pass).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.nn.functional as F


def elementwise(d: torch.Tensor, kind: str, delta: float = 1.0) -> torch.Tensor:
    if kind == 'mse':
        return d * d
    if kind == 'huber':
        ad = d.abs()
        return torch.where(ad <= delta, 0.5 * d * d, delta * (ad - 0.5 * delta))
    raise ValueError(kind)


def scalar_td_loss(q: torch.Tensor, actions: torch.Tensor, rewards: torch.Tensor,
                   dones: torch.Tensor, q_next_target: torch.Tensor,
                   q_next_online: Optional[torch.Tensor] = None, gamma: float = 0.99,
                   kind: str = 'mse', delta: float = 1.0,
                   weights: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Returns (loss, |td_error|). ``q_next_online`` given => Double DQN."""
    a = actions.long().view(-1, 1)
    q_sa = q.gather(1, a).squeeze(1)
    with torch.no_grad():
        sel = q_next_online if q_next_online is not None else q_next_target
        a_star = sel.argmax(dim=1, keepdim=True)
        nxt = q_next_target.gather(1, a_star).squeeze(1)
        y = rewards.float() + gamma * (1.0 - dones.float()) * nxt
    d = q_sa - y
    per = elementwise(d, kind, delta)
    if weights is not None:
        per = per * weights
    return per.mean(), d.detach().abs()


def categorical_projection(p_next: torch.Tensor, rewards: torch.Tensor, dones: torch.Tensor,
                           gamma: float, v_min: float, v_max: float) -> torch.Tensor:
    """Project r + gamma*z onto the fixed support (Bellemare et al. 2017). p_next: [B, N]."""
    B, N = p_next.shape
    z = torch.linspace(v_min, v_max, N, device=p_next.device)
    dz = (v_max - v_min) / (N - 1)
    tz = (rewards.float().view(B, 1) + gamma * (1.0 - dones.float().view(B, 1)) * z.view(1, N))
    tz = tz.clamp(v_min, v_max)
    b = (tz - v_min) / dz
    lo = b.floor().long()
    hi = b.ceil().long()
    m = torch.zeros(B, N, device=p_next.device)
    eq = (lo == hi).float()
    m.scatter_add_(1, lo, p_next * (hi.float() - b + eq))
    m.scatter_add_(1, hi, p_next * (b - lo.float()))
    return m


def c51_loss(logits: torch.Tensor, actions: torch.Tensor, rewards: torch.Tensor,
             dones: torch.Tensor, logits_next_target: torch.Tensor,
             logits_next_online: Optional[torch.Tensor], gamma: float, v_min: float,
             v_max: float, weights: Optional[torch.Tensor] = None):
    """logits: [B, A, N]. Returns (loss, per-sample cross-entropy)."""
    B, A, N = logits.shape
    z = torch.linspace(v_min, v_max, N, device=logits.device)
    with torch.no_grad():
        p_t = torch.softmax(logits_next_target.float(), dim=-1)
        sel = logits_next_online if logits_next_online is not None else logits_next_target
        q_sel = (torch.softmax(sel.float(), dim=-1) * z).sum(-1)
        a_star = q_sel.argmax(dim=1)
        p_next = p_t[torch.arange(B, device=logits.device), a_star]
        m = categorical_projection(p_next, rewards, dones, gamma, v_min, v_max)
    logp = F.log_softmax(logits.float(), dim=-1)[torch.arange(B, device=logits.device), actions.long()]
    per = -(m * logp).sum(-1)
    pr = per.detach().clone()
    if weights is not None:
        per = per * weights
    return per.mean(), pr
