"""Flat parameter storage.

Every parameter of a Q-network lives in ONE contiguous fp32 buffer so that
the optimizer is a single fused kernel, the data-parallel gradient exchange
is a single (or a few bucketed) collective(s), and the target update is one
device-to-device copy / Polyak kernel (reference: per-variable TF ops,
`/root/reference/src/network.py:69-75,198-202,251-252`).

Layout: L2-regularised weights first (so the optimizer kernel applies the
decoupled ``reg_param * w`` term to ``flat[:reg_end]`` with no mask), then the
rest. Each tensor starts on a 64-element (256 B) boundary for vector loads.
Tensor shapes are the TF layouts (conv HWIO, dense [in, out]).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Tuple

import torch

from .arch import ArchSpec

ALIGN = 64


def _round_up(n: int, a: int = ALIGN) -> int:
    return (n + a - 1) // a * a


class FlatLayout:
    def __init__(self, arch: ArchSpec):
        specs = arch.param_specs()
        reg = set(arch.reg_names())
        ordered = [s for s in specs if s[0] in reg] + [s for s in specs if s[0] not in reg]
        self.names: List[str] = []
        self.shapes: Dict[str, Tuple[int, ...]] = {}
        self.kinds: Dict[str, str] = {}
        self.offsets: Dict[str, int] = {}
        off = 0
        self.reg_end = 0
        for name, shape, kind in ordered:
            self.names.append(name)
            self.shapes[name] = tuple(shape)
            self.kinds[name] = kind
            self.offsets[name] = off
            off += _round_up(math.prod(shape))
            if name in reg:
                self.reg_end = off
        self.total = off
        self.tf_order = [s[0] for s in specs]

    def numel(self, name: str) -> int:
        return math.prod(self.shapes[name])

    def views(self, flat: torch.Tensor) -> Dict[str, torch.Tensor]:
        return {n: flat[self.offsets[n]:self.offsets[n] + self.numel(n)].view(self.shapes[n])
                for n in self.names}


def truncated_normal_(t: torch.Tensor, std: float, generator: Optional[torch.Generator] = None):
    """TF ``truncated_normal_initializer``: resample draws beyond 2 sigma."""
    flat = t.view(-1)
    buf = torch.empty(flat.numel(), dtype=torch.float32)
    buf.normal_(0.0, std, generator=generator)
    bad = buf.abs() > 2 * std
    while bool(bad.any()):
        n = int(bad.sum())
        buf[bad] = torch.empty(n).normal_(0.0, std, generator=generator)
        bad = buf.abs() > 2 * std
    flat.copy_(buf)
    return t


class ParamStore:
    """One network's parameters as views over a flat fp32 buffer."""

    def __init__(self, arch: ArchSpec, device='cpu', flat: Optional[torch.Tensor] = None):
        self.arch = arch
        self.layout = FlatLayout(arch)
        self.device = torch.device(device)
        if flat is None:
            flat = torch.zeros(self.layout.total, dtype=torch.float32, device=self.device)
        assert flat.numel() == self.layout.total and flat.dtype == torch.float32
        self.flat = flat
        self.tensors = self.layout.views(self.flat)

    def init_(self, seed: Optional[int] = None):
        """Reference init (`network.py:269-270,341-342`): trunc-normal(0.01) weights, zero biases.

        Noisy layers use the factorised-Gaussian init of Fortunato et al.
        """
        g = torch.Generator().manual_seed(seed if seed is not None else torch.seed() % (2 ** 63))
        host = torch.zeros(self.layout.total, dtype=torch.float32)
        views = self.layout.views(host)
        for name in self.layout.tf_order:
            kind, v = self.layout.kinds[name], views[name]
            layer = name.rsplit('/', 1)[0]
            dense = next((d for d in self.arch.dense_layers() if d.name == layer), None)
            if dense is not None and dense.noisy:
                bound = 1.0 / math.sqrt(dense.fin)
                if kind in ('w', 'b'):
                    v.uniform_(-bound, bound, generator=g)
                else:
                    v.fill_(self.arch.noisy_sigma0 / math.sqrt(dense.fin))
            elif kind == 'w':
                truncated_normal_(v, 0.01, g)
            else:
                v.zero_()
        self.flat.copy_(host.to(self.device))
        return self

    def copy_from(self, other: 'ParamStore'):
        self.flat.copy_(other.flat)

    def state_dict(self) -> Dict[str, torch.Tensor]:
        return {n: self.tensors[n].detach().cpu().clone() for n in self.layout.tf_order}

    def load_state_dict(self, sd: Dict[str, torch.Tensor], strict: bool = True):
        for n in self.layout.tf_order:
            if n not in sd:
                if strict:
                    raise KeyError('missing parameter %s' % n)
                continue
            src = torch.as_tensor(sd[n])
            if tuple(src.shape) != self.layout.shapes[n]:
                raise ValueError('shape mismatch for %s: %s vs %s' % (n, tuple(src.shape), self.layout.shapes[n]))
            self.tensors[n].copy_(src.to(self.flat.device, torch.float32))
