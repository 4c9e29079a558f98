"""`Network`: the model/graph-builder layer (reference C4/C5/C8,
`/root/reference/src/network.py:13-254`).

The reference builds a TF graph and hands the agent graph handles
(`q_output`, `target_q_output`, `train_op`, `target_update_ops`,
`global_step`). Here those handles are methods over device-resident flat
buffers:

  reference handle            -> here
  q_output                    -> q_values(x)
  target_q_output             -> target_q_values(x)
  train_op (+global_step++)   -> train_step(batch)  (= compute_grads + apply_grads)
  target_update_ops           -> update_target()    (one D2D copy / Polyak kernel)
  global_step                 -> global_step (device int64, advanced by the optimizer)

Target parameters are replicated per rank (reference default,
`network.py:216-225`). With `--disable_target_replication` (reference
`network.py:226-231`: target on the PS) rank 0 owns the target: under sync DP
the learner broadcasts rank 0's target after every target sync (`Learner`),
under `--async_ps` the parameter server holds it and workers pull it when it
changes (`parallel/async_ps.py`), and checkpoints carry ``target/*``.
"""
from __future__ import annotations

import logging
from typing import Dict, Optional

import torch

from .. import optim
from ..ops import kernels
from . import torch_net
from .arch import ArchSpec, arch_from_config
from .executor import TorchExecutor
from .params import ParamStore

log = logging.getLogger(__name__)


def resolve_device(config) -> torch.device:
    dev = getattr(config, 'device', 'auto')
    if dev == 'auto':
        dev = 'cuda' if torch.cuda.is_available() else 'cpu'
    if dev == 'cuda':
        return torch.device('cuda', torch.cuda.current_device())
    return torch.device(dev)


def make_executor(arch: ArchSpec, layout, config, device: torch.device):
    backend = getattr(config, 'backend', 'auto')
    kw = dict(input_scale=config.input_scale, loss=config.loss, huber_delta=config.huber_delta,
              double_dqn=config.double_dqn)
    if device.type == 'cuda' and backend in ('auto', 'hip') and not arch.is_conv:
        # MLP nets (the reference SimpleNetwork): one fused fp32 kernel per SGD step
        from ..ops.mlp_executor import HipMlpExecutor, supports_mlp
        if supports_mlp(arch):
            return HipMlpExecutor(arch, layout, **kw)
        if backend == 'hip':
            raise RuntimeError('HIP MLP executor does not support %s' % (arch,))
    if device.type == 'cuda' and backend in ('auto', 'hip') and arch.is_conv:
        from ..ops.executor import make_hip_executor, supports
        if supports(arch):
            # --dtype: bf16 / fp16 (16-bit MFMA builds) or fp32 (the reference's precision: the
            # fp32-MFMA build of the same kernels, _C_f32)
            from ..ops.tuning import KernelTuning
            return make_hip_executor(arch, layout, dtype=config.dtype,
                                     tuning=KernelTuning.parse(getattr(config, 'kernel_tuning', '')), **kw)
        if backend == 'hip':
            raise RuntimeError('HIP executor does not support %s' % (arch,))
        log.warning('HIP conv executor does not support this architecture (network=%s input=%s atoms=%s); '
                    'falling back to the torch (MIOpen) executor, which is several times slower',
                    arch.network, tuple(arch.input_shape), getattr(arch, 'atoms', None))
    return TorchExecutor(arch, layout, **kw)


class Network:
    def __init__(self, arch: ArchSpec, config, device=None, num_replicas: int = 1,
                 ps_device=None, worker_device=None):
        self.arch = arch
        self.config = config
        self.device = torch.device(device) if device is not None else resolve_device(config)
        self.num_replicas = num_replicas
        self.ps_device, self.worker_device = ps_device, worker_device
        self.online = ParamStore(arch, self.device).init_(config.seed)
        self.target = ParamStore(arch, self.device)
        self.target.copy_from(self.online)
        self.layout = self.online.layout
        self.grad = torch.zeros_like(self.online.flat)
        self.optimizer = optim.make_optimizer(config, self.layout, self.device)
        self.global_step = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.executor = make_executor(arch, self.layout, config, self.device)
        nz = torch_net.noise_size(arch)
        self.noise = torch.zeros(nz, device=self.device) if nz else None
        self.noise_target = torch.zeros(nz, device=self.device) if nz else None
        self.last_loss = torch.zeros(1, device=self.device)
        # noisy nets on the HIP executor: the online weights' packed / effective buffers are
        # kept mixed under self.noise. Samples come from a device Philox stream seeded by the
        # run seed (identical on every DP rank); after each update the fused optimizer derives
        # the sigma gradients from the mu gradients under self.noise, mixes in the next sample
        # (drawn with the next target sample, one launch) and makes it current — so the
        # learner and the device actors launch no mix for the online net.
        self._premixed = bool(nz) and hasattr(self.executor, 'premix')
        if self._premixed:
            self.noise_next = torch.zeros_like(self.noise)
            seed = int(config.seed) if getattr(config, 'seed', None) is not None else 0
            self.noise_rng = torch.tensor([(seed * 0x9E3779B1 + 0x6E6F) & 0x7fffffffffff, 0], dtype=torch.int64,
                                          device=self.device)
            self.executor.draw_noise(self.noise, self.noise_target, self.noise_rng)
            self.executor.premix(self.online.flat, self.noise)
            # the target runs forward only: its fc layer may keep mu / sigma fragments and mix the
            # noise in its forward (HipExecutor.set_factorised)
            if hasattr(self.executor, 'set_factorised'):
                self.executor.set_factorised(self.target.flat)
            self.executor.premix(self.target.flat, self.noise_target)

    # -------------------------------------------------------------- factory
    @staticmethod
    def create_network(config, input_shape, num_actions, num_replicas=1, ps_device=None,
                       worker_device=None, device=None) -> 'Network':
        """Reference factory signature (`network.py:35-57`)."""
        arch = arch_from_config(config, input_shape, num_actions)
        return Network(arch, config, device=device, num_replicas=num_replicas,
                       ps_device=ps_device, worker_device=worker_device)

    # ------------------------------------------------------------ inference
    def _to_dev(self, x):
        if not torch.is_tensor(x):
            import numpy as np
            x = torch.from_numpy(np.ascontiguousarray(np.asarray(x)))
        return x.to(self.device, non_blocking=True)

    def q_values(self, x) -> torch.Tensor:
        return self.executor.q_values(self.online.flat, self._to_dev(x), self.noise)

    def target_q_values(self, x) -> torch.Tensor:
        return self.executor.q_values(self.target.flat, self._to_dev(x), self.noise_target)

    def reset_noise(self, generator=None):
        """Fresh online and target noise samples now (torch RNG when a generator is given)."""
        if self.noise is None:
            return
        if self._premixed and generator is None:
            self.executor.draw_noise(self.noise, self.noise_target, self.noise_rng)
        else:
            self.noise.normal_(generator=generator)
            self.noise_target.normal_(generator=generator)
        if self._premixed:
            self.executor.premix(self.online.flat, self.noise)
            self.executor.premix(self.target.flat, self.noise_target)

    def begin_step_noise(self):
        """Noise for one learner step. Premixed executors: nothing to do (both samples were
        drawn by the previous ``apply_grads``); otherwise fresh online and target samples."""
        if self.noise is not None and not self._premixed:
            self.reset_noise()

    def fuses_update(self, target_freq: Optional[int]) -> bool:
        """True when ``apply_grads(.., target_freq)`` is ONE optimizer+pack launch (which can
        also draw the next uniform minibatch, ``next_sample``)."""
        ex = self.executor
        return (target_freq is not None and self.online.flat.is_cuda and self.optimizer.backend != 'torch'
                and hasattr(ex, 'update_and_pack') and (self._premixed or not getattr(ex, 'noisy', False)))

    def fuses_sigma_grads(self, target_freq: Optional[int]) -> bool:
        """True when ``apply_grads(.., target_freq)`` runs the fused noisy optimizer, which
        derives dL/dsigma itself (so ``compute_grads(sigma_grads=False)`` may skip it)."""
        return (self._premixed and target_freq is not None and self.online.flat.is_cuda
                and self.optimizer.backend != 'torch')

    # ------------------------------------------------------------- training
    def compute_grads(self, batch: Dict[str, torch.Tensor], acting: Optional[dict] = None, split: bool = False,
                      sigma_grads: bool = True, lowrank: Optional[dict] = None, defer_fc: bool = False,
                      det_wgrad: bool = False, defer_wgrad: bool = False):
        """Loss + gradient into ``self.grad``. ``split=True`` returns ``(loss, prio, tail)``: when
        ``tail`` is not None only the dense-layer gradients (``dense_range()``) are final and
        ``tail()`` queues the rest of the backward (see HipExecutor.loss_and_grad). ``defer_fc``:
        the fc weight / bias gradient is left to the next fused ``apply_grads`` (it forms them
        inside the optimizer launch; ``HipExecutor.can_defer_fc``). ``det_wgrad``: the conv weight
        gradients stay as deterministic partials the next fused ``apply_grads`` sums
        (``HipExecutor.can_det_wgrad``). ``defer_wgrad`` (with ``defer_fc``): the grouped conv /
        output-layer weight gradients are computed by the next fused ``apply_grads`` beside the
        fc update (``HipExecutor.can_defer_wgrad``)."""
        kw = {}
        if defer_wgrad:
            kw['defer_wgrad'] = True
        if defer_fc:
            kw['defer_fc'] = True
        if det_wgrad:
            kw['det_wgrad'] = True
        if self._premixed and not sigma_grads:
            # the fused noisy optimizer follows: it derives dL/dsigma itself, and the next samples
            # are drawn by a launch of this backward (no noise launch of their own)
            kw['sigma_grads'] = False
            kw['draw_noise'] = (self.noise_next, self.noise_target, self.noise_rng)
            self._noise_drawn = True
        if acting is not None:     # fused acting (HIP executor): the actors' step rides along
            kw['acting'] = acting
        can_split = split and hasattr(self.executor, 'supports_fused_acting')
        if can_split:
            kw['split'] = True
            if lowrank is not None:      # DP: fc weight gradient from all-gathered factors
                kw['lowrank'] = lowrank
        out = self.executor.loss_and_grad(self.online.flat, self.target.flat, batch, self.grad,
                                          self.noise, self.noise_target, **kw)
        loss, prio = out[0], out[1]
        tail = out[2] if can_split else None
        self.last_loss = loss
        return (loss, prio, tail) if split else (loss, prio)

    def dense_range(self):
        """[0, X): the longest prefix of the flat buffer holding only dense-layer parameters
        (the L2-regularised dense weights come first, `models/params.py`). Its gradient is final
        before the conv backward runs, so data parallelism reduces it first."""
        lay = self.layout
        dense = {n for n in lay.names if not any(n.startswith(c.name + '/') for c in self.arch.convs)}
        end = lay.total
        for n in sorted(lay.names, key=lambda n: lay.offsets[n]):
            if n not in dense:
                end = lay.offsets[n]        # 64-element aligned: whole collective vectors
                break
        return 0, end

    def apply_grads(self, grad_scale: float = 1.0, target_freq: Optional[int] = None, next_sample=None,
                    grad: Optional[torch.Tensor] = None, repack: bool = True) -> bool:
        """Optimizer step (global_step += 1 inside it) + executor repack.

        target_freq: also do the hard target sync (target <- online when the new
        global_step % target_freq == 0, device predicate) inside those same two
        launches. Returns True when it was fused that way; otherwise the caller
        still owes the target update (``hard_target_update``). next_sample: ``(spec, B)`` — the
        fused launch also draws the next uniform minibatch (only honoured when it returns True).
        grad: the gradient buffer to apply (default ``self.grad``; the xgmi parameter server passes
        a worker's peer-written slot). repack=False (the parameter server, which never runs the
        network): the optimizer step only; the caller calls ``refresh_packed`` before the packed
        copies are used again."""
        ex = self.executor
        g = self.grad if grad is None else grad
        fuse = (target_freq is not None and self.online.flat.is_cuda and self.optimizer.backend != 'torch'
                and hasattr(ex, 'packed'))
        if fuse and hasattr(ex, 'update_and_pack') and (self._premixed or not getattr(ex, 'noisy', False)):
            # optimizer + repack + hard target sync: one launch (noisy nets: + the mix of the
            # next online noise sample, drawn here)
            kw = {}
            if self._premixed:
                # next online sample (+ the next step's target sample); the optimizer derives
                # dL/dsigma under the current one, mixes the next one in and makes it current.
                # The samples were drawn during compute_grads (its fc dgrad launch) when it knew
                # this fused update follows; the optimizer then advances the stream's counter.
                if getattr(self, '_noise_drawn', False):
                    kw['noise_rng'] = self.noise_rng
                    self._noise_drawn = False
                else:
                    self.executor.draw_noise(self.noise_next, self.noise_target, self.noise_rng)
                kw.update(noise=self.noise_next, grad_noise=self.noise, noise_dst=self.noise,
                          target_noise=self.noise_target)
            ex.update_and_pack(self.optimizer, self.online.flat, g, grad_scale, self.global_step,
                               target=self.target.flat, target_freq=int(target_freq), next_sample=next_sample, **kw)
            return True
        assert next_sample is None or not fuse, 'next_sample needs the fused optimizer+pack launch'
        assert not (hasattr(ex, 'pending_fc') and ex.pending_fc()), \
            'compute_grads(defer_fc / det_wgrad) needs the fused optimizer+pack update'
        if fuse:
            self.optimizer.step(self.online.flat, g, grad_scale, self.global_step,
                                target=self.target.flat, target_freq=int(target_freq))
            # (noisy nets: every consumer re-mixes + repacks under its own noise sample)
            if not getattr(ex, 'noisy', False):
                ex.repack(self.online.flat, target=self.target.flat, step=self.global_step,
                          freq=int(target_freq))
            return True
        self.optimizer.step(self.online.flat, g, grad_scale, self.global_step)
        if repack:
            self._repack()
        return False

    def _repack(self):
        if hasattr(self.executor, 'repack'):
            self.executor.repack(self.online.flat)

    def refresh_packed(self):
        """Rebuild the executor's packed copies of online AND target from their fp32 masters
        (after a broadcast or restore; noisy nets re-mix under their bound noise samples)."""
        if hasattr(self.executor, 'repack'):
            self.executor.repack(self.online.flat)
            self.executor.repack(self.target.flat)

    def hard_target_update(self, step: Optional[torch.Tensor] = None, freq: int = 1):
        """target <- online when step % freq == 0 (device predicate); fp32 master and the
        executor's packed copy move in ONE launch."""
        ex = self.executor
        if hasattr(ex, 'packed'):
            pt, po = ex.packed(self.target.flat), ex.packed(self.online.flat)
            kernels.target_update(self.target.flat, self.online.flat, 1.0, step, freq,
                                  extra=(pt.view(torch.float32), po.view(torch.float32)))
            if self._premixed:              # noisy: the target's fragments follow its own noise
                ex.premix(self.target.flat, self.noise_target)
        else:
            kernels.target_update(self.target.flat, self.online.flat, 1.0, step, freq)

    def sync_target_copy(self, tau: float, step: Optional[torch.Tensor] = None, freq: int = 1):
        """Executor-side refresh after ``target <- online`` (packed bf16 weights)."""
        if hasattr(self.executor, 'sync_target'):
            self.executor.sync_target(self.target.flat, self.online.flat, tau, step, freq)

    def train_step(self, batch: Dict[str, torch.Tensor], grad_scale: float = 1.0):
        loss, prio = self.compute_grads(batch)
        self.apply_grads(grad_scale)
        return loss, prio

    def update_target(self, tau: Optional[float] = None):
        tau = self.config.target_update_tau if tau is None else tau
        kernels.target_update(self.target.flat, self.online.flat, min(1.0, tau))
        self.sync_target_copy(min(1.0, tau))

    def total_loss(self) -> float:
        """Reference `loss` summary value: TD loss + reg_param * sum 0.5||w||^2."""
        reg = torch_net.reg_loss(self.layout, self.online.flat)
        return float(self.last_loss) + self.config.reg_param * float(reg)

    # ----------------------------------------------------------- checkpoint
    def _flats(self) -> Dict[str, torch.Tensor]:
        """The flat buffers a checkpoint holds (see ``state_dict``)."""
        fl = {'online': self.online.flat, 'step': self.global_step, 'beta': self.optimizer.beta_powers}
        for i, sl in enumerate(self.optimizer.slots):
            fl['slot%d' % i] = sl
        if self.config.disable_target_replication:
            fl['target'] = self.target.flat
        return fl

    def snapshot(self):
        """Device copies of the checkpointed buffers, taken on a side stream in stream order after
        the work queued so far (the next step waits for the copies, ~tens of us of D2D, not for a
        host transfer). Returns ``(snap, event)``: ``state_dict_from(snap)`` after ``event`` —
        a writer thread can do the D2H and the file write off the training thread."""
        fl = self._flats()
        if not self.online.flat.is_cuda:
            return {k: v.detach().clone() for k, v in fl.items()}, None
        dev = self.online.flat.device
        main = torch.cuda.current_stream(dev)
        side = getattr(self, '_ckpt_stream', None)
        if side is None:
            side = self._ckpt_stream = torch.cuda.Stream(device=dev)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            snap = {k: v.detach().clone() for k, v in fl.items()}
            ev = torch.cuda.Event()
            ev.record(side)
        main.wait_stream(side)        # the next update must not overwrite a buffer mid-copy
        for v in snap.values():
            v.record_stream(side)
        return snap, ev

    def state_dict_from(self, fl: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        """TF-named CPU tensors from flat buffers (``_flats()`` or a ``snapshot``)."""
        lay = self.layout
        host = {k: v.detach().cpu() for k, v in fl.items()}
        views = lay.views(host['online'])
        sd = {n: views[n].clone() for n in lay.tf_order}
        opt = self.optimizer
        for i, suffix in enumerate(opt.slot_names()):
            for name, v in lay.views(host['slot%d' % i]).items():
                sd['%s/%s' % (name, suffix)] = v.clone()
        if opt.name == 'adam':
            sd['beta1_power'] = host['beta'][0:1].view(()).clone()
            sd['beta2_power'] = host['beta'][1:2].view(()).clone()
        sd['global_step'] = host['step'].view(()).clone()
        if 'target' in host:
            tv = lay.views(host['target'])
            sd.update({'target/' + n: tv[n].clone() for n in lay.tf_order})
        return sd

    def state_dict(self) -> Dict[str, torch.Tensor]:
        return self.state_dict_from(self._flats())

    def load_state_dict(self, sd: Dict[str, torch.Tensor]):
        self.online.load_state_dict(sd)
        self.optimizer.load_state_dict(sd)
        if 'global_step' in sd:
            self.global_step.fill_(int(sd['global_step']))
        tsd = {k[len('target/'):]: v for k, v in sd.items() if k.startswith('target/')}
        if tsd:
            self.target.load_state_dict(tsd)
        self.refresh_packed()
