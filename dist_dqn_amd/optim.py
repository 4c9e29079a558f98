"""TF-0.x-exact optimizers over a flat parameter buffer.

The reference picks `tf.train.*Optimizer(learning_rate=lr)` at
`/root/reference/src/network.py:169-177,184` and applies it with
``minimize(var_list=params, global_step)`` at `:198-202`. These are the TF
library update rules, including TF's slot initial values
(RMSProp ``ms = 1``, Adagrad/FTRL accumulators = 0.1) which differ from
``torch.optim``.

Two implementations of the same math:
  * `apply_torch` — a handful of vectorised torch ops on the flat buffers
    (CPU path, oracle);
  * the fused HIP kernel `csrc/kernels/optim.hip` (one launch for all
    parameters, decoupled L2 on ``flat[:reg_end]``, 1/world gradient
    averaging folded in), used when the buffers live on the GPU.
Slot tensors and their TF checkpoint names: `slot_names()`.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch

from .models.params import FlatLayout

OPT_IDS = {'sgd': 0, 'momentum': 1, 'rmsprop': 2, 'adam': 3, 'adagrad': 4, 'adadelta': 5, 'ftrl': 6}
RMSPROP_NO_MOMENTUM = 7    # kernel variant: rmsprop with momentum 0 never reads the mom slot


def kernel_op(opt) -> int:
    """Kernel op id of an optimizer (RMSProp at the TF default momentum 0 skips its mom read:
    bit-identical update, one fp32 slot less of HBM traffic per step)."""
    if opt.name == 'rmsprop' and float(opt.hp['rms_mom']) == 0.0:
        return RMSPROP_NO_MOMENTUM
    return OPT_IDS[opt.name]

# (slot suffixes in TF checkpoint naming, initial value)
_SLOTS = {
    'sgd': [],
    'momentum': [('Momentum', 0.0)],
    'rmsprop': [('RMSProp', 1.0), ('RMSProp_1', 0.0)],
    'adam': [('Adam', 0.0), ('Adam_1', 0.0)],
    'adagrad': [('Adagrad', 0.1)],
    'adadelta': [('Adadelta', 0.0), ('Adadelta_1', 0.0)],
    'ftrl': [('Ftrl', 0.1), ('Ftrl_1', 0.0)],
}


class FlatOptimizer:
    def __init__(self, name: str, layout: FlatLayout, device, lr: float, reg_param: float = 0.0,
                 momentum: float = 0.9, rmsprop_decay: float = 0.95, rmsprop_momentum: float = 0.0,
                 rmsprop_eps: float = 1e-10, adam_b1: float = 0.9, adam_b2: float = 0.999,
                 adam_eps: float = 1e-8, adadelta_rho: float = 0.95, adadelta_eps: float = 1e-8,
                 backend: str = 'auto'):
        if name not in OPT_IDS:
            raise RuntimeError('Unsupported optimizer {}'.format(name))
        self.name = name
        self.layout = layout
        self.device = torch.device(device)
        self.lr = float(lr)
        self.reg_param = float(reg_param)
        self.hp = dict(momentum=momentum, rho=rmsprop_decay, rms_mom=rmsprop_momentum,
                       rms_eps=rmsprop_eps, b1=adam_b1, b2=adam_b2, adam_eps=adam_eps,
                       ad_rho=adadelta_rho, ad_eps=adadelta_eps)
        n = layout.total
        self.slots: List[torch.Tensor] = [torch.full((n,), init, dtype=torch.float32, device=self.device)
                                          for _, init in _SLOTS[name]]
        # Adam's beta powers are TF non-slot variables (beta1_power, beta2_power).
        self.beta_powers = torch.tensor([adam_b1, adam_b2], dtype=torch.float32, device=self.device)
        self.backend = backend
        # HIP kernels: arrival tickets (1 + 16 sub-tickets, 128 B apart) and, word 1, the slot flag
        self.ticket = (torch.zeros(17 * 32, dtype=torch.int32, device=self.device)
                       if self.device.type == 'cuda' else None)
        self._slots_on = False

    @property
    def defers_slots(self) -> bool:
        """Momentum-0 RMSProp on the HIP kernels stores its ``mom`` slot (TF ``RMSProp_1``, never
        read by the update) only on steps after ``request_slots(True)``: one fp32 write per
        parameter less per step. The checkpoint manager raises the flag one step before a save."""
        return (self.device.type == 'cuda' and self.backend != 'torch' and self.name == 'rmsprop'
                and float(self.hp['rms_mom']) == 0.0)

    def request_slots(self, on: bool = True):
        """Store the deferred slot on the following steps (device flag read by every launch)."""
        if self.defers_slots and bool(on) != self._slots_on:
            self.ticket[1].fill_(1 if on else 0)
            self._slots_on = bool(on)

    # ------------------------------------------------------------------ API
    def slot_names(self) -> List[str]:
        return [s for s, _ in _SLOTS[self.name]]

    def state_dict(self) -> Dict[str, torch.Tensor]:
        """TF-named slot tensors: '<var>/<Slot>' plus beta powers for Adam."""
        out = {}
        for suffix, buf in zip(self.slot_names(), self.slots):
            for name, v in self.layout.views(buf).items():
                out['%s/%s' % (name, suffix)] = v.detach().cpu().clone()
        if self.name == 'adam':
            out['beta1_power'] = self.beta_powers[0:1].view(()).cpu().clone()
            out['beta2_power'] = self.beta_powers[1:2].view(()).cpu().clone()
        return out

    def load_state_dict(self, sd: Dict[str, torch.Tensor]):
        for suffix, buf in zip(self.slot_names(), self.slots):
            for name, v in self.layout.views(buf).items():
                key = '%s/%s' % (name, suffix)
                if key in sd:
                    v.copy_(torch.as_tensor(sd[key]).to(buf.device))
        if self.name == 'adam' and 'beta1_power' in sd:
            self.beta_powers[0] = float(sd['beta1_power'])
            self.beta_powers[1] = float(sd['beta2_power'])

    def step(self, param: torch.Tensor, grad: torch.Tensor, grad_scale: float = 1.0,
             global_step: Optional[torch.Tensor] = None, target: Optional[torch.Tensor] = None,
             target_freq: int = 1):
        """param -= update(grad * grad_scale + reg * w) in place; global_step += 1.

        target (HIP path): also copy the updated params into it when the new
        global_step % target_freq == 0 (fused hard target sync)."""
        if param.is_cuda and self.backend != 'torch':
            from .ops import kernels
            kernels.optimizer_step(self, param, grad, grad_scale, global_step, target, target_freq)
        else:
            self.apply_torch(param, grad, grad_scale)
            if global_step is not None:
                global_step += 1

    # --------------------------------------------------------------- oracle
    def apply_torch(self, w: torch.Tensor, g_in: torch.Tensor, grad_scale: float = 1.0):
        hp, lr, n = self.hp, self.lr, self.name
        g = g_in.float() * grad_scale if grad_scale != 1.0 else g_in.float().clone()
        if self.reg_param != 0.0:
            re = self.layout.reg_end
            g[:re] += self.reg_param * w[:re]
        if n == 'sgd':
            w.sub_(lr * g)
        elif n == 'momentum':
            acc, = self.slots
            acc.mul_(hp['momentum']).add_(g)
            w.sub_(lr * acc)
        elif n == 'rmsprop':
            ms, mom = self.slots
            ms.mul_(hp['rho']).addcmul_(g, g, value=1.0 - hp['rho'])
            mom.mul_(hp['rms_mom']).add_(lr * g / torch.sqrt(ms + hp['rms_eps']))
            w.sub_(mom)
        elif n == 'adam':
            m, v = self.slots
            b1p, b2p = self.beta_powers[0], self.beta_powers[1]
            lr_t = lr * torch.sqrt(1 - b2p) / (1 - b1p)
            m.mul_(hp['b1']).add_(g, alpha=1 - hp['b1'])
            v.mul_(hp['b2']).addcmul_(g, g, value=1 - hp['b2'])
            w.sub_(lr_t * m / (torch.sqrt(v) + hp['adam_eps']))
            self.beta_powers.mul_(torch.tensor([hp['b1'], hp['b2']], device=self.beta_powers.device))
        elif n == 'adagrad':
            acc, = self.slots
            acc.addcmul_(g, g)
            w.sub_(lr * g / torch.sqrt(acc))
        elif n == 'adadelta':
            accum, accum_upd = self.slots
            rho, eps = hp['ad_rho'], hp['ad_eps']
            accum.mul_(rho).addcmul_(g, g, value=1 - rho)
            upd = torch.sqrt(accum_upd + eps) / torch.sqrt(accum + eps) * g
            accum_upd.mul_(rho).addcmul_(upd, upd, value=1 - rho)
            w.sub_(lr * upd)
        elif n == 'ftrl':
            accum, linear = self.slots
            new_accum = accum + g * g
            linear.add_(g - (torch.sqrt(new_accum) - torch.sqrt(accum)) / lr * w)
            quadratic = torch.sqrt(new_accum) / lr
            w.copy_(torch.where(linear.abs() > 0.0, -linear / quadratic, torch.zeros_like(w)))
            accum.copy_(new_accum)
        return w


def make_optimizer(config, layout: FlatLayout, device, backend: str = 'auto') -> FlatOptimizer:
    return FlatOptimizer(config.optimizer, layout, device, lr=config.lr, reg_param=config.reg_param,
                         momentum=config.momentum, rmsprop_decay=config.rmsprop_decay, backend=backend)
