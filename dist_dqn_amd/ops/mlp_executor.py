"""Fused HIP executor for MLP Q-networks (`csrc/kernels/mlp.hip`).

The reference `SimpleNetwork` (`/root/reference/src/network.py:258-313`: in -> 20
tanh -> 20 tanh -> A, the CartPole net) and any plain dense chain of <= 4 layers
with widths <= 64. One launch computes the whole SGD-step gradient (online and
target forwards, TD loss, backward, batch-reduced weight gradients); one launch
computes Q for acting. fp32 throughout: these layers are far below an MFMA tile.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from . import _ext

_ACT = {None: 0, 'tanh': 1, 'relu': 2}
MAX_LAYERS, MAX_WIDTH, THREADS = 4, 64, 128


def supports_mlp(arch) -> bool:
    if arch.is_conv or arch.dueling or arch.distributional or arch.noisy:
        return False
    layers = arch.dense_layers()
    if not 1 <= len(layers) <= MAX_LAYERS:
        return False
    if any(d.fin > MAX_WIDTH or d.fout > MAX_WIDTH for d in layers):
        return False
    return True


class HipMlpExecutor:
    name = 'hip'
    compute_dtype = 'fp32'

    def __init__(self, arch, layout, input_scale: float = 1.0, loss: str = 'mse', huber_delta: float = 1.0,
                 double_dqn: bool = False, **_):
        assert supports_mlp(arch), 'HIP MLP executor: unsupported architecture'
        self.ext = _ext.load(required=True)
        self.arch, self.layout = arch, layout
        self.input_scale = float(input_scale)
        self.huber = loss == 'huber'
        self.delta = float(huber_delta)
        self.double = bool(double_dqn)
        layers = arch.dense_layers()
        self.L = len(layers)
        self.A = arch.num_actions
        pad = lambda v: list(v) + [0] * (MAX_LAYERS - len(v))
        fin = [d.fin for d in layers]
        fout = [d.fout for d in layers]
        self.D = fin[0]
        self.sw = max(fout)
        hs = sum(fin) + fout[-1]
        ds = max(sum(fout), 2 * self.sw)
        self.Hs = hs | 1                  # odd row strides: lane rows hit distinct LDS banks
        self.Ds = ds | 1
        self.P = layout.total
        self._ints_tail = (pad(fin) + pad(fout) + pad([_ACT[d.act] for d in layers])
                           + pad([layout.offsets[d.name + '/w'] for d in layers])
                           + pad([layout.offsets[d.name + '/b'] for d in layers]))
        lds = self.ext.mlp_lds_bytes([self.P, self.Hs, self.Ds])
        if lds > 160 * 1024:
            raise RuntimeError('MLP too large for the single-workgroup kernel (%d B LDS)' % lds)
        self._ws: Dict[tuple, dict] = {}

    def _ints(self, B: int):
        return [self.L, self.A, self.P, self.Hs, self.Ds, self.sw, B, int(self.double), int(self.huber)] + \
            self._ints_tail

    def _ws_for(self, B: int, dev) -> dict:
        key = (B, dev.index)
        ws = self._ws.get(key)
        if ws is None:
            f32 = dict(dtype=torch.float32, device=dev)
            ws = {'loss': torch.zeros(1, **f32), 'prio': torch.zeros(B, **f32)}
            self._ws[key] = ws
        return ws

    def _states(self, x: torch.Tensor) -> torch.Tensor:
        x = x.reshape(x.shape[0], -1)
        assert x.shape[1] == self.D, 'MLP input width %d != %d' % (x.shape[1], self.D)
        if x.dtype != torch.float32 or not x.is_contiguous():
            x = x.float().contiguous()
        return x

    def forward(self, flat: torch.Tensor, x: torch.Tensor, noise=None) -> torch.Tensor:
        x = self._states(x)
        B = x.shape[0]
        q = torch.empty(B, self.A, dtype=torch.float32, device=x.device)
        self.ext.mlp(0, self._ints(B), [flat.data_ptr(), 0, x.data_ptr()] + [0] * 9 + [q.data_ptr()],
                     [self.delta, self.input_scale], flat)
        return q

    def q_values(self, flat, x, noise=None):
        return self.forward(flat, x)

    def loss_and_grad(self, online: torch.Tensor, target: torch.Tensor, batch: Dict[str, torch.Tensor],
                      grad_out: torch.Tensor, noise=None, noise_target=None, acting: Optional[dict] = None,
                      split: bool = False):
        assert acting is None, 'fused acting is a conv-network feature'
        s, ns = self._states(batch['states']), self._states(batch['next_states'])
        B = s.shape[0]
        dev = s.device
        assert online.is_contiguous() and target.is_contiguous() and grad_out.numel() == self.P
        act = batch['actions']
        if act.dtype != torch.int32:
            act = act.to(torch.int32)
        act = act.contiguous()
        cols = [batch[k].float().contiguous() for k in ('rewards', 'dones', 'gammas')]
        assert act.numel() == B and all(c.numel() == B for c in cols)
        wts = batch.get('weights')
        if wts is not None:
            wts = wts.float().contiguous()
        ws = self._ws_for(B, dev)
        self.ext.mlp(1, self._ints(B),
                     [online.data_ptr(), target.data_ptr(), s.data_ptr(), ns.data_ptr(), act.data_ptr()]
                     + [c.data_ptr() for c in cols]
                     + [wts.data_ptr() if wts is not None else 0, ws['loss'].data_ptr(), ws['prio'].data_ptr(),
                        grad_out.data_ptr(), 0],
                     [self.delta, self.input_scale], online)
        out = (ws['loss'], ws['prio'])
        return out + (None,) if split else out
