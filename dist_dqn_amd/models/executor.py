"""Executors: how a Q-network's forward / loss+gradient is computed.

`TorchExecutor` — PyTorch ops + autograd over the flat buffer (CPU path and
numerics oracle). The fused HIP executor lives in `dist_dqn_amd/ops/executor.py`
and implements the same two methods with hand-written CDNA4 kernels.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch

from . import torch_net
from .arch import ArchSpec
from .params import FlatLayout


class TorchExecutor:
    name = 'torch'
    compute_dtype = 'fp32'

    def __init__(self, arch: ArchSpec, layout: FlatLayout, input_scale: float = 1.0,
                 loss: str = 'mse', huber_delta: float = 1.0, double_dqn: bool = False, oracle: bool = False):
        """oracle=True: every op in PyTorch, the TD loss included (the numerics reference the HIP
        kernels are tested against); otherwise the TD loss on cuda tensors runs the fused
        td_loss kernel (the `simple` MLP's GPU training path)."""
        self.arch, self.layout = arch, layout
        self.input_scale = input_scale
        self.loss_kind, self.delta, self.double = loss, huber_delta, double_dqn
        self.oracle = bool(oracle)

    def forward(self, flat: torch.Tensor, x: torch.Tensor, noise: Optional[torch.Tensor] = None):
        with torch.no_grad():
            return torch_net.forward(self.arch, flat, self.layout, x, self.input_scale, noise)

    def q_values(self, flat, x, noise=None):
        return torch_net.q_from_logits(self.arch, self.forward(flat, x, noise))

    def loss_and_grad(self, online: torch.Tensor, target: torch.Tensor, batch: Dict[str, torch.Tensor],
                      grad_out: torch.Tensor, noise: Optional[torch.Tensor] = None,
                      noise_target: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        """Writes dLoss/dflat into grad_out; returns (loss [1], |td| or CE per sample [B])."""
        arch = self.arch
        flat = online.detach().requires_grad_(True)
        out = torch_net.forward(arch, flat, self.layout, batch['states'], self.input_scale, noise)
        with torch.no_grad():
            nt = torch_net.forward(arch, target, self.layout, batch['next_states'], self.input_scale, noise_target)
            no = (torch_net.forward(arch, online, self.layout, batch['next_states'], self.input_scale, noise)
                  if self.double else None)
        from ..ops.td import td_loss
        loss, prio = td_loss(out, batch['actions'], batch['rewards'], batch['dones'], batch['gammas'], nt, no,
                             batch.get('weights'), self.loss_kind, self.delta, arch.distributional,
                             arch.v_min, arch.v_max, pure_torch=self.oracle)
        g, = torch.autograd.grad(loss, flat)
        grad_out.copy_(g)
        return loss.detach().view(1), prio
