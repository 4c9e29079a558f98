"""PyTorch oracle executor for an `ArchSpec`.

Plain PyTorch ops on the TF-layout views of the flat buffer; autograd gives
the gradient as ONE flat tensor (via `Unflatten`). It is the numerics
reference the HIP kernels are tested against and the executor used on CPU
(CartPole, gloo tests). Reference layers: `/root/reference/src/network.py:298-309`
(MLP) and `:389-424` (conv + bias + ReLU + SAME max-pool, HWC flatten).
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import torch
import torch.nn.functional as F

from .arch import ArchSpec, DenseSpec
from .params import FlatLayout


class Unflatten(torch.autograd.Function):
    """flat -> tuple of TF-shaped views; backward packs the grads into one flat tensor."""

    @staticmethod
    def forward(ctx, flat, layout: FlatLayout):
        ctx.layout = layout
        views = layout.views(flat)
        return tuple(views[n] for n in layout.names)

    @staticmethod
    def backward(ctx, *grads):
        lay = ctx.layout
        ref = next(g for g in grads if g is not None)
        out = torch.zeros(lay.total, dtype=ref.dtype, device=ref.device)
        for n, g in zip(lay.names, grads):
            if g is not None:
                o = lay.offsets[n]
                out[o:o + lay.numel(n)].copy_(g.reshape(-1))
        return out, None


def unflatten(flat: torch.Tensor, layout: FlatLayout) -> Dict[str, torch.Tensor]:
    if flat.requires_grad:
        return dict(zip(layout.names, Unflatten.apply(flat, layout)))
    return layout.views(flat)


def noise_size(arch: ArchSpec) -> int:
    """Number of factorised-noise scalars (eps_in + eps_out per noisy layer)."""
    return sum(d.fin + d.fout for d in arch.dense_layers() if d.noisy)


def _scale_noise(x):
    return x.sign() * x.abs().sqrt()


def _dense(x, p, d: DenseSpec, noise: Optional[torch.Tensor], noff: int):
    w, b = p[d.name + '/w'], p[d.name + '/b']
    if d.noisy and noise is not None:
        ei = _scale_noise(noise[noff:noff + d.fin])
        eo = _scale_noise(noise[noff + d.fin:noff + d.fin + d.fout])
        w = w + p[d.name + '/w_sigma'] * torch.outer(ei, eo)
        b = b + p[d.name + '/b_sigma'] * eo
    y = x @ w + b
    if d.act == 'relu':
        y = F.relu(y)
    elif d.act == 'tanh':
        y = torch.tanh(y)
    return y


def forward(arch: ArchSpec, flat: torch.Tensor, layout: FlatLayout, x: torch.Tensor,
            input_scale: float = 1.0, noise: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Returns Q [B, A] (scalar heads) or logits [B, A, atoms] (distributional)."""
    p = unflatten(flat, layout)
    h = x.to(torch.float32)
    if input_scale != 1.0:
        h = h * input_scale
    if arch.is_conv:
        h = h.permute(0, 3, 1, 2)                       # NHWC -> NCHW
        for c in arch.convs:
            t, bt, l, r = c.pads()
            if t or bt or l or r:
                h = F.pad(h, (l, r, t, bt))
            w = p[c.name + '/w'].permute(3, 2, 0, 1)    # HWIO -> OIHW
            h = F.relu(F.conv2d(h, w, p[c.name + '/b'], stride=c.stride))
            if c.pool:
                t, bt, l, r = c.pool_pads()
                if t or bt or l or r:
                    h = F.pad(h, (l, r, t, bt), value=float('-inf'))
                h = F.max_pool2d(h, 2, 2)
        h = h.permute(0, 2, 3, 1).reshape(h.shape[0], -1)  # TF HWC flatten order
    noff = 0
    for d in arch.trunk:
        h = _dense(h, p, d, noise, noff)
        noff += d.fin + d.fout if d.noisy else 0
    B, A, N = h.shape[0], arch.num_actions, arch.atoms
    if arch.dueling:
        v = h
        for d in arch.value:
            v = _dense(v, p, d, noise, noff)
            noff += d.fin + d.fout if d.noisy else 0
        a = h
        for d in arch.head:
            a = _dense(a, p, d, noise, noff)
            noff += d.fin + d.fout if d.noisy else 0
        a = a.view(B, A, N)
        out = v.view(B, 1, N) + a - a.mean(dim=1, keepdim=True)
    else:
        for d in arch.head:
            h = _dense(h, p, d, noise, noff)
            noff += d.fin + d.fout if d.noisy else 0
        out = h.view(B, A, N)
    return out if arch.distributional else out.view(B, A)


def reg_loss(layout: FlatLayout, flat: torch.Tensor) -> torch.Tensor:
    """Sum of tf.nn.l2_loss over the regularised weights: 0.5 * ||w||^2."""
    return 0.5 * (flat[:layout.reg_end].float() ** 2).sum()


def q_from_logits(arch: ArchSpec, out: torch.Tensor) -> torch.Tensor:
    if not arch.distributional:
        return out
    z = torch.linspace(arch.v_min, arch.v_max, arch.atoms, device=out.device)
    return (torch.softmax(out.float(), dim=-1) * z).sum(-1)


def support(arch: ArchSpec, device) -> torch.Tensor:
    return torch.linspace(arch.v_min, arch.v_max, arch.atoms, device=device)


def sample_noise(arch: ArchSpec, device, generator=None) -> Optional[torch.Tensor]:
    n = noise_size(arch)
    if n == 0:
        return None
    return torch.randn(n, device=device, generator=generator)


__all__ = ['forward', 'reg_loss', 'q_from_logits', 'noise_size', 'sample_noise', 'support', 'math']
