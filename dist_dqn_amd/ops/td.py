"""TD-loss op: fused HIP kernel on the GPU (`csrc/kernels/td_loss.hip`),
torch oracle (`models/losses.py`) on the CPU. Differentiable w.r.t. the
online Q values / logits; the kernel emits dL/dQ in its forward launch and
backward only scales it.
"""
from __future__ import annotations

from typing import Optional

import torch

from ..models import losses
from . import _ext


class _TDLossHip(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, actions, rewards, dones, gammas, next_t, next_o, weights, kind, delta, c51, vmin, vmax):
        ext = _ext.load(required=True)
        B = q.shape[0]
        loss = torch.empty(1, dtype=torch.float32, device=q.device)
        dq = torch.empty_like(q, dtype=torch.float32)
        prio = torch.empty(B, dtype=torch.float32, device=q.device)
        qf = q.float().contiguous()
        args = (qf, next_t.float().contiguous(), None if next_o is None else next_o.float().contiguous(),
                actions.to(torch.int32).contiguous(), rewards.float().contiguous(), dones.float().contiguous(),
                gammas.float().contiguous(), None if weights is None else weights.float().contiguous(),
                loss, dq, prio)
        if c51:
            ext.td_loss_c51(*args, float(vmin), float(vmax))
        else:
            ext.td_loss_scalar(*args, kind == 'huber', float(delta))
        ctx.save_for_backward(dq)
        ctx.mark_non_differentiable(prio)
        return loss, prio

    @staticmethod
    def backward(ctx, g_loss, g_prio):
        dq, = ctx.saved_tensors
        return (dq * g_loss,) + (None,) * 12


def td_loss(out: torch.Tensor, actions, rewards, dones, gammas, next_t, next_o=None,
            weights: Optional[torch.Tensor] = None, kind: str = 'mse', delta: float = 1.0,
            distributional: bool = False, v_min: float = -10.0, v_max: float = 10.0, pure_torch: bool = False):
    """Returns (mean loss [scalar], per-sample priority [B]). pure_torch: the torch oracle on any
    device (the numerics reference of the HIP kernels)."""
    if out.is_cuda and not pure_torch:
        loss, prio = _TDLossHip.apply(out, actions, rewards, dones, gammas, next_t, next_o, weights, kind, delta,
                                      distributional, v_min, v_max)
        return loss.view(()), prio
    if distributional:
        return losses.c51_loss(out, actions, rewards, dones, next_t, next_o, gammas.view(-1, 1), v_min, v_max,
                               weights)
    return losses.scalar_td_loss(out, actions, rewards, dones, next_t, next_o, gammas, kind, delta, weights)
