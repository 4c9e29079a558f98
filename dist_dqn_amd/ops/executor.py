"""Fused HIP executor: the Q-network forward / backward on hand-written
gfx950 kernels (`csrc/kernels/qnet.hip`), bf16 MFMA with fp32 accumulation
and fp32 master weights / gradients / optimizer state.

One learner step = (after the replay sample+gather kernels)
  conv1 fwd | conv2 fwd | conv3 fwd | fc fwd     (online(s), target(s')[, online(s')] as grid.z instances)
  head+TD-loss+head-backward                     (one workgroup)
  fc wgrad | fc dgrad | conv3 wgrad | conv3 dgrad | conv2 wgrad | conv2 dgrad | conv1 wgrad
i.e. 11 kernels for the whole network + loss + gradient (the torch path runs
~60 kernels for the same work). Weights are re-packed from the fp32 master
buffer into bf16 MFMA B-fragments once per optimizer step (`repack`), and the
target's packed copy is refreshed by a predicated copy when the target syncs.

Supported: `nature` convs (84x84x4 uint8 frames), plain or dueling heads,
scalar (MSE/Huber) or C51 distributional (csrc/kernels/rainbow.hip), noisy
dense layers (factorised Gaussian: effective weights mixed on the GPU, then
packed; sigma gradients split from the mu gradients), Double DQN, PER weights.
The reference `cnn` (SAME convs + max-pools) runs on the per-sample fused
kernels of csrc/kernels/cnn.hip (`HipCnnExecutor`). `simple` uses torch.
"""
from __future__ import annotations

import os
from typing import Dict, Optional, Tuple

import torch

from . import _ext

_KIND = dict(C1=1, C2=2, C3=3, DFWD=4, DF32=5, DDGRAD=6, D3=7, D2=8, F1=9, HW=11, DLR=12)


def supports(arch) -> bool:
    if arch.network not in ('nature', 'cnn'):
        return False
    if arch.distributional and arch.atoms > 64:     # one wave64 lane per atom
        return False
    if tuple(arch.input_shape) != (84, 84, 4):
        return False
    return True


class _Job:
    __slots__ = ('src_off', 'K', 'N', 'dst_off', 'dst_N16', 'nt_off', 'ks_off', 'mode', 'p0', 'p1', 'p2')

    def __init__(self, **kw):
        for k in self.__slots__:
            setattr(self, k, kw.get(k, 0))

    def ints(self):
        return [self.src_off, self.K, self.N, self.dst_off, self.dst_N16, self.nt_off, self.ks_off, self.mode,
                self.p0, self.p1, self.p2, 0]

    def threads(self):
        if self.mode == 3:
            return self.K
        return ((self.K + 31) // 32) * ((self.N + 15) // 16) * 64


def _frag_elems(K, N):
    return ((K + 31) // 32) * ((N + 15) // 16) * 512


class HipExecutor:
    name = 'hip'
    compute_dtype = 'bf16'
    consumes_slots = True       # conv1 reads the replay frame ring through [B, 4] slot tables

    def __init__(self, arch, layout, dtype: str = 'bf16', input_scale: float = 1.0, loss: str = 'mse',
                 huber_delta: float = 1.0, double_dqn: bool = False, tuning=None):
        assert supports(arch), 'HIP executor: unsupported architecture'
        # fp16 (--dtype=fp16) / fp32 (--dtype=fp32, the reference's training precision): the same
        # kernels built with -DDQN_F16 (fp16 MFMA, static loss scale inside the kernels) or
        # -DDQN_F32 (fp32 MFMA); everything else (fp32 master state, layouts) is shared
        assert dtype in ('bf16', 'fp16', 'fp32'), dtype
        self.fp16 = dtype == 'fp16'
        self.compute_dtype = dtype
        self.act_dtype = {'bf16': torch.bfloat16, 'fp16': torch.float16, 'fp32': torch.float32}[dtype]
        self.esz = torch.tensor([], dtype=self.act_dtype).element_size()   # bytes per packed / act element
        self.fs = 4 // self.esz                  # act_t slots of one fp32 value inside the packed buffer
        self.ext = _ext.load(required=True, variant={'bf16': '', 'fp16': 'f16', 'fp32': 'f32'}[dtype])
        self.arch, self.layout = arch, layout
        from .tuning import KernelTuning
        self.tuning = tuning if tuning is not None else KernelTuning()
        self.input_scale = float(input_scale)
        self.huber = loss == 'huber'
        self.delta = float(huber_delta)
        self.double = bool(double_dqn)
        self.A = arch.num_actions
        self.dueling = arch.dueling
        self.dist = arch.distributional
        self.atoms = arch.atoms if self.dist else 1
        self.NO = self.A * self.atoms          # output-layer width (advantage / plain head)
        self.noisy = arch.noisy
        self._eff: Dict[int, torch.Tensor] = {}
        fc = arch.value[0] if self.dueling else arch.head[0]
        self.HID = fc.fout
        self.HH = 2 * self.HID if self.dueling else self.HID
        self.FLAT = arch.flat_features
        # C51 dL/dlogits rows (dout16 [B][KD]): logits at [0, NO), dueling value at [VO, VO + atoms)
        self.c51_VO = (self.NO + 31) // 32 * 32
        self.c51_KD = self.c51_VO + ((self.atoms + 31) // 32 * 32 if self.dueling else 0)
        # noisy C51 nets: a flat marked with ``set_factorised`` (the learner's target) keeps its fc
        # weights packed as separate mu / sigma fragments that change only at a target sync; its fc
        # forward mixes the per-step noise itself (qnet.hip fc_fwd_fz_kernel: X Wmu + f(eps_out) *
        # ((X * f(eps_in)) Wsigma)), so the optimizer launch neither reads the target's fc weights nor
        # re-packs them every step (~10 bytes / fc weight of its ~60). Opt-in (KernelTuning.tfact):
        # measured on Rainbow, the optimizer launch 58.4 -> 53.2 us but the fc forward 10.5 -> 20.0 us
        # (the target's fragments, written only at a sync, are read cold from HBM, twice the bytes), so
        # 7.29k -> 7.04k SGD steps/s on one box (gpurun_out/r5aa, r5ab)
        self.tfact = (self.noisy and self.dist and dtype != 'fp32' and arch.network == 'nature'
                      and bool(self.tuning.tfact))
        self._fact: Dict[int, torch.Tensor] = {}      # flat ptr -> sigma fragments (packed layout)
        self._fact_pk: Dict[int, int] = {}            # packed ptr -> flat ptr (factorised flats)
        self._fz_noise: Dict[int, torch.Tensor] = {}  # flat ptr -> the noise its packed fc bias holds
        self._plan_packing()
        self._packed: Dict[int, torch.Tensor] = {}
        self._ws: Dict[Tuple[int, int], dict] = {}
        self.two_stream = False
        self.fused_trunk = True     # conv1..conv3 in one per-sample kernel (trunk.hip)
        self.fold_head = True       # training: fc forward + scalar head in one launch (fc_head.hip)
        # the fold's spin mode (its dH-tile blocks wait for their group's tail: every block resident);
        # off when several processes share the GPU (the one-GPU DP rehearsals: another rank's spinning
        # collective blocks can hold the CUs a tail needs -- the waits then expire, learner.py)
        self.fold_spin = True
        # fc + conv3 dgrads in one launch (dgrad_chain_kernel; 2: + conv2). Opt-in: measured 12.1 us vs
        # 4.96 + 5.16 us for the two launches (the waits and the write-through stores cost more than the
        # launch boundary saves; 14.34k / 13.99k / 14.50k steps/s for 1 / 2 / 0, profiles/r4_dgrad_chain_ab.jsonl)
        self.chain_dgrad = 0
        self._fc_zero = None        # int32 counters the next fc forward launch zeroes (the chain's)
        self.grouped_wgrad = True   # every layer's weight gradient in ONE launch after the dgrad chain
        # (round 2 measured the fc + output-layer members on a parallel graph branch beside the dgrad
        # chain: 12.0k -> 9.9k steps/s, the captured fork / join costs more than the overlap gains)
        # fused optimizer+pack grid cap (one block per 32x64 tile; grid-stride beyond it)
        self.opt_max_grid = 2048
        self.trunk_prof = None      # int64 [ninst*B*8] phase-timestamp buffer (scripts/probe_trunk.py)
        self.head_prof = None       # int64 [32] head phase stamps (scripts/probe_head.py)
        self.fold_prof = None       # int64 [blocks * 8] fused fc + head stamps (scripts/probe_fold.py)
        self.cnn_prof = None        # (fwd, bwd) int64 [blocks * 8] cnn kernel stamps (scripts/probe_cnn.py)
        self._events = {}

    # ------------------------------------------------------------ packing
    def _plan_packing(self):
        lay, arch = self.layout, self.arch
        off = 0
        jobs = []
        self.poff = {}

        def add(key, K, N, entries):
            nonlocal off
            self.poff[key] = off
            N16 = (N + 15) // 16
            for e in entries:
                jobs.append(_Job(dst_off=off, dst_N16=N16, **e))
            off += _frag_elems(K, N)
            off = (off + 255) // 256 * 256

        for c in arch.convs:
            K = c.k * c.k * c.cin
            add(c.name + '/fwd', K, c.cout, [dict(src_off=lay.offsets[c.name + '/w'], K=K, N=c.cout, mode=0)])
            if c.name != arch.convs[0].name:
                Kd = c.k * c.k * c.cout
                add(c.name + '/dgrad', Kd, c.cin,
                    [dict(src_off=lay.offsets[c.name + '/w'], K=Kd, N=c.cin, mode=1, p0=c.k * c.k, p1=c.cin,
                          p2=c.cout)])
        F, H = self.FLAT, self.HID
        if self.dueling:
            fcs = [('value/fcl', 0), ('advantage/fcl', H)]
        else:
            fcs = [('fcl', 0)]
        add('fc/fwd', F, self.HH, [dict(src_off=lay.offsets[n + '/w'], K=F, N=H, nt_off=o // 16, mode=0)
                                    for n, o in fcs])
        add('fc/dgrad', self.HH, F, [dict(src_off=lay.offsets[n + '/w'], K=H, N=F, ks_off=o // 32, mode=2, p0=H)
                                      for n, o in fcs])
        hw = 'advantage/output/w' if self.dueling else 'output/w'
        hb = 'advantage/output/b' if self.dueling else 'output/b'
        if not self.dist:
            # scalar head: output-layer fragments for the head kernel's MFMA Q tiles
            add('head/w', H, self.NO, [dict(src_off=lay.offsets[hw], K=H, N=self.NO, mode=0)])
            if self.dueling:
                add('head/v', H, self.atoms, [dict(src_off=lay.offsets['value/output/w'], K=H, N=self.atoms,
                                                   mode=0)])
        else:
            # C51: the output layer as ONE combined GEMM over the whole hidden row [value | advantage]:
            # Wc [HH][KD] = [[0, Wv at column VO], [W_adv, 0]] (block diagonal), so every instance's
            # logits AND value logits come from one igemm launch (rows of KD = dout16's columns)
            wc = [dict(src_off=lay.offsets[hw], K=H, N=self.NO, ks_off=(H // 32) if self.dueling else 0, mode=0)]
            if self.dueling:
                wc.append(dict(src_off=lay.offsets['value/output/w'], K=H, N=self.atoms, nt_off=self.c51_VO // 16,
                               mode=0))
            add('head/wc', self.HH, self.c51_KD, wc)
            # C51: dgrad fragments of the output layer(s) for the dH igemm, K' = [logits | value]:
            # dH = dout16 [B][KD] . (plain / advantage W^T into h's advantage half, Wv^T into the value half)
            dg = [dict(src_off=lay.offsets[hw], K=self.NO, N=H, nt_off=H // 16 if self.dueling else 0, mode=2,
                       p0=self.NO)]
            if self.dueling:
                dg.append(dict(src_off=lay.offsets['value/output/w'], K=self.atoms, N=H, ks_off=self.c51_VO // 32,
                               mode=2, p0=self.atoms))
            add('head/dgrad', self.c51_KD, self.HH, dg)
        # concatenated fc bias (fp32: self.fs act_t slots per float)
        self.poff['fc/bias'] = off
        for n, o in fcs:
            jobs.append(_Job(src_off=lay.offsets[n + '/b'], K=H, dst_off=off + self.fs * o, mode=3))
        off += self.fs * self.HH
        off = (off + 255) // 256 * 256
        if self.dist:
            # C51: the combined output layer's bias row (fp32): logits bias | pad | value bias at VO
            self.poff['head/bias'] = off
            jobs.append(_Job(src_off=lay.offsets[hb], K=self.NO, dst_off=off, mode=3))
            if self.dueling:
                jobs.append(_Job(src_off=lay.offsets['value/output/b'], K=self.atoms, dst_off=off + self.fs * self.c51_VO,
                                 mode=3))
            off += self.fs * self.c51_KD
            off = (off + 255) // 256 * 256
        self.packed_elems = off
        self.jobs = jobs
        self._jobs_dev: Dict[torch.device, torch.Tensor] = {}
        self._max_threads = max(j.threads() for j in jobs)
        self._plan_noisy()
        self._plan_update()

    def _plan_update(self):
        """Work list of the fused optimizer+pack kernel (optim.hip optim_pack_kernel): 32x64
        tiles of every packed weight tensor (forward fragments + its dgrad fragments), then
        2048-element chunks of everything else (with the fc bias fp32 copy).

        Noisy nets: each noisy mu tile / chunk also carries its sigma tensor (updated in the
        same thread; sigma tensors get no items of their own) and the noise offsets, so the
        packed fragments (and the fp32 ``eff`` values of everything read in fp32: all but the
        big fc weights) are mu + sigma * f(eps_in) f(eps_out) under the bound noise sample."""
        lay = self.layout
        fwd, dg, copy = {}, {}, {}
        for j in self.jobs:
            if j.mode == 0:
                fwd[j.src_off] = j
            elif j.mode in (1, 2):
                dg[j.src_off] = j
            else:
                copy[j.src_off] = j
        nz, sig = {}, set()
        if self.noisy:
            noff = 0
            for d in self.arch.dense_layers():
                if d.noisy:
                    nz[lay.offsets[d.name + '/w']] = (lay.offsets[d.name + '/w_sigma'], noff, noff + d.fin)
                    nz[lay.offsets[d.name + '/b']] = (lay.offsets[d.name + '/b_sigma'], -1, noff + d.fin)
                    sig |= {lay.offsets[d.name + '/w_sigma'], lay.offsets[d.name + '/b_sigma']}
                    noff += d.fin + d.fout
        fc_names = [('value/fcl', 0), ('advantage/fcl', self.HID)] if self.dueling else [('fcl', 0)]
        fc_w = {lay.offsets[n + '/w'] for n, _ in fc_names if n + '/w' in lay.offsets}
        # fused fc weight gradient (optim.hip FcFuse): the dH column of each fc weight / bias tensor
        fc_col = {}
        for n, col in fc_names:
            if n + '/w' in lay.offsets:
                fc_col[lay.offsets[n + '/w']] = col
                fc_col[lay.offsets[n + '/b']] = col
        items = []
        for src, f in sorted(fwd.items()):
            d = dg.get(src)
            so, ei, eo = nz.get(src, (-1, -1, -1))
            # eff bit 0: store the fp32 effective values; bit 1: factorised target fc tile (tfact)
            eff = int(self.noisy and src not in fc_w) | (2 if self.tfact and src in fc_w else 0)
            fcc = fc_col.get(src, -1)
            assert fcc < 0 or (f.K % 8 == 0 and f.N % 8 == 0)
            for k0 in range(0, f.K, 32):
                for n0 in range(0, f.N, 64):
                    items.append([0, src, f.K, f.N, k0, n0, f.dst_off, f.dst_N16, f.nt_off, f.ks_off,
                                  d.mode if d else 0, d.dst_off if d else 0, d.dst_N16 if d else 0,
                                  d.nt_off if d else 0, d.ks_off if d else 0, d.p1 if d else 0, so, ei, eo, eff,
                                  fcc, -1, 0, 0, 0])
        for name in lay.names:
            off, n = lay.offsets[name], lay.numel(name)
            if off in fwd or off in sig:
                continue
            c = copy.get(off)
            so, _, eo = nz.get(off, (-1, -1, -1))
            fcc = fc_col.get(off, -1)
            assert fcc < 0 or n <= 512, 'fused fc bias gradient: one chunk of <= 512 values'
            for s0 in range(0, n, 2048):
                cnt = min(2048, n - s0)
                items.append([1, off + s0, cnt, 0, 0, 0, (c.dst_off + self.fs * s0) if c else -1] + [0] * 9
                             + [so + s0 if so >= 0 else -1, -1, eo + s0 if so >= 0 else -1, int(self.noisy), fcc,
                                -1, 0, 0, 0])
        self.upd_items = items
        self._upd_dev: Dict[torch.device, torch.Tensor] = {}
        # (x ptr, dh ptr, rows) of a step whose fc weight gradient the next update_and_pack forms
        self._fc_pending = None
        # (members, dims, scales) of a step whose grouped conv / output-layer weight gradients the
        # next update_and_pack computes in its first launch (loss_and_grad(defer_wgrad=True))
        self._wg_pending = None
        self._wg_plans: Dict[tuple, tuple] = {}
        # 128-row chunks per conv weight-gradient tile of the fused launch (KernelTuning.wg_conv_chunks)
        self.wg_conv_chunks = self.tuning.conv_chunks(self.arch.network, self.compute_dtype)
        # data parallelism (learner.py): the transport whose exchange channel the fused update launch
        # uses to sum the dependent jobs' gradients over every rank (parallel/xgmi.py dpx_launch); None:
        # one process
        self.dp_exchange = None
        # (job table, partial buffer ptr) of a step whose conv weight gradients the next
        # update_and_pack sums from the grouped wgrad's deterministic partials
        self._parts_pending = None
        self._det: Dict[tuple, dict] = {}
        self._bound: Dict[int, torch.Tensor] = {}   # flat ptr -> noise its packed/eff buffers reflect
        self._dummies: Dict[torch.device, tuple] = {}

    def _upd_jobs(self, dev):
        jobs = self._upd_dev.get(dev)
        if jobs is None:
            ints = [v for it in self.upd_items for v in it]
            assert len(ints) == len(self.upd_items) * self.ext.UPD_JOB_INTS
            jobs = torch.tensor(ints, dtype=torch.int32, device=dev)
            self._upd_dev[dev] = jobs
        return jobs

    def _eff_for(self, key: int, like: torch.Tensor) -> torch.Tensor:
        eff = self._eff.get(key)
        if eff is None:
            eff = torch.zeros_like(like)
            self._eff[key] = eff
        return eff

    def _mix_pack(self, flat: torch.Tensor, noise: Optional[torch.Tensor], eff: torch.Tensor, p: torch.Tensor):
        """Noisy nets: ONE launch (optim_pack_kernel<-1>, no update) writing the packed fragments
        and the fp32 effective values of ``flat`` under ``noise`` (None: zero noise, eff = mu)."""
        dev = flat.device
        d = self._dummies.get(dev)
        if d is None:
            from ..models.torch_net import noise_size
            d = (torch.zeros(2, dtype=torch.float32, device=dev), torch.zeros(17 * 32, dtype=torch.int32, device=dev),
                 torch.zeros(1, dtype=torch.int64, device=dev),
                 torch.zeros(noise_size(self.arch), dtype=torch.float32, device=dev))
            self._dummies[dev] = d
        if noise is None:
            noise = d[3]
        assert noise.numel() >= d[3].numel() and noise.dtype == torch.float32
        k = flat.data_ptr()
        tsg = self._fact.get(k)
        if tsg is not None:          # factorised flat: p gets the mu fragments, tsg the sigma ones
            self._fz_noise[k] = noise
        self.ext.optim_pack(-1, flat, flat, flat, flat, d[0], d[1], 0.0, 0.0, 0, 1.0, d[2], [0.0] * 9,
                            self._upd_jobs(dev), p, None, None, 1, self.opt_max_grid, noise, eff, None, None, [], [],
                            [], None, None, None, None, [], 0, tsg=tsg.data_ptr() if tsg is not None else 0)

    def draw_noise(self, out0: torch.Tensor, out1: Optional[torch.Tensor], rng: torch.Tensor):
        """Standard normals into out0 (and out1) from the device Philox state ``rng`` (one launch)."""
        self.ext.noise_normal(out0, out1, rng)

    def set_factorised(self, flat: torch.Tensor) -> bool:
        """Mark ``flat`` (a target net: forward only) for the factorised noisy fc forward (see
        ``tfact``); its packed copy is re-made by the next ``premix`` / ``effective``. Returns whether
        it applies to this executor."""
        if not self.tfact:
            return False
        k = flat.data_ptr()
        if k not in self._fact:
            self._fact[k] = torch.zeros(self.packed_elems, dtype=self.act_dtype, device=flat.device)
            self._fact_pk[self._packed_for(k, flat).data_ptr()] = k
            self._bound.pop(k, None)
        return True

    def premix(self, flat: torch.Tensor, noise: torch.Tensor):
        """Bind ``noise`` to ``flat``: its packed / eff buffers now hold the effective weights
        under that sample, and stay so (the noisy fused optimizer re-mixes after each update),
        so consumers using that same noise tensor (learner online instance, device actors,
        q_values) launch no mix of their own."""
        assert self.noisy
        k = flat.data_ptr()
        self._mix_pack(flat, noise, self._eff_for(k, flat), self._packed_for(k, flat))
        self._bound[k] = noise

    def update_and_pack(self, opt, flat: torch.Tensor, grad: torch.Tensor, grad_scale: float,
                        global_step: torch.Tensor, target: Optional[torch.Tensor] = None, target_freq: int = 1,
                        noise: Optional[torch.Tensor] = None, grad_noise: Optional[torch.Tensor] = None,
                        noise_dst: Optional[torch.Tensor] = None, next_sample=None,
                        target_noise: Optional[torch.Tensor] = None, noise_rng: Optional[torch.Tensor] = None,
                        fc=None, pack: bool = True):
        """Optimizer step + repack in ONE launch (+ the hard target sync under the device
        predicate when ``target`` is given). Noisy nets: ``noise`` (the next sample for this
        flat) is mixed in and bound (see ``premix``); the target's packed copy is not written
        (the target is re-mixed under its own noise every step). ``grad_noise``: derive the
        sigma gradients from the mu-slot gradients under that sample (the one the forward
        used) instead of reading them; ``noise_dst``: the kernel's last block copies ``noise``
        there, and ``noise_dst`` becomes the bound noise. ``next_sample``: a
        ``DeviceReplay.next_sample_spec`` dict — one extra block of this launch draws the next
        step's minibatch (uniform, or prioritized after writing this step's priorities).
        ``target_noise`` (noisy nets): the target is mixed + packed under it in the same launch
        and bound to it (no target mix launch next step). ``noise_rng``: the stream whose next
        samples ``loss_and_grad(draw_noise=...)`` drew this step; the last block advances its
        counter. ``fc``: the pending fused fc weight gradient of ``loss_and_grad(defer_fc=True)``
        (default: taken from this executor; the launch forms dW = X^T dH and the fc bias gradient
        from those rows instead of reading them from ``grad``). ``pack=False``: the update only, no packed
        fragments written (a caller that never runs the network until it repacks). Returns True."""
        from ..optim import kernel_op
        dev = flat.device
        assert pack or (self._wg_pending is None and not self.noisy), 'pack=False: plain fused update only'
        if self._wg_pending is not None:
            return self._update_split(opt, flat, grad, grad_scale, global_step, target, target_freq, noise, grad_noise,
                                      noise_dst, next_sample, target_noise, noise_rng, fc)
        jobs, part = self._upd_jobs(dev), 0
        if self._parts_pending is not None:
            (jobs, part), self._parts_pending = self._parts_pending, None
        hp = opt.hp
        s0 = opt.slots[0] if len(opt.slots) > 0 else flat
        s1 = opt.slots[1] if len(opt.slots) > 1 else flat
        if getattr(opt, 'ticket', None) is None or opt.ticket.device != dev or opt.ticket.numel() < 17 * 32:
            opt.ticket = torch.zeros(17 * 32, dtype=torch.int32, device=dev)   # 1 + 16 sub-tickets, 128 B apart
        eff = teff = tpk = None
        if self.noisy:
            assert noise is not None and noise.dtype == torch.float32
            k = flat.data_ptr()
            p, eff = self._packed_for(k, flat), self._eff_for(k, flat)
            pt = None
            if target_noise is not None:
                assert target is not None and target_noise.dtype == torch.float32
                tk = target.data_ptr()
                tpk, teff = self._packed_for(tk, target), self._eff_for(tk, target)
        else:
            p = self.packed(flat)
            pt = self.packed(target) if target is not None else None
        self.ext.optim_pack(kernel_op(opt), flat, grad, s0, s1, opt.beta_powers, opt.ticket, float(opt.lr),
                            float(opt.reg_param), int(opt.layout.reg_end), float(grad_scale), global_step,
                            [float(hp['momentum']), float(hp['rho']), float(hp['rms_mom']), float(hp['rms_eps']),
                             float(hp['b1']), float(hp['b2']), float(hp['adam_eps']), float(hp['ad_rho']),
                             float(hp['ad_eps'])], jobs, p, target, pt, int(target_freq), self.opt_max_grid,
                            noise, eff, grad_noise, noise_dst,
                            (list(next_sample['spec']) + [int(next_sample['B'])]
                             if next_sample is not None and next_sample['kind'] == 'uniform' else []),
                            (list(next_sample['p']) if next_sample is not None and next_sample['kind'] == 'per' else []),
                            (list(next_sample['f']) if next_sample is not None and next_sample['kind'] == 'per' else []),
                            target_noise, teff, tpk, noise_rng, self._take_fc(fc), part, tsg=self._tsg_arg(target, target_noise),
                            no_pack=not pack)
        if self.noisy:
            self._bound[flat.data_ptr()] = noise_dst if noise_dst is not None else noise
            if target_noise is not None:
                self._bound[target.data_ptr()] = target_noise
        return True

    def prepare_update(self, opt, flat: torch.Tensor):
        """Allocate what ``update_and_pack`` creates on first use (the device job table, the
        optimizer's arrival ticket, the packed buffer), so a first call inside a graph capture does
        no host-to-device copy."""
        dev = flat.device
        self._upd_jobs(dev)
        if getattr(opt, 'ticket', None) is None or opt.ticket.device != dev or opt.ticket.numel() < 17 * 32:
            opt.ticket = torch.zeros(17 * 32, dtype=torch.int32, device=dev)
        self.packed(flat)

    def _tsg_arg(self, target, target_noise) -> int:
        """The optimizer launch's factorised-target argument: the target's sigma fragments (written at
        a sync step) when the launch mixes a factorised target under ``target_noise`` (now its bias
        noise, which the target forward reads), else 0."""
        if target is None or target_noise is None:
            return 0
        tsg = self._fact.get(target.data_ptr())
        if tsg is None:
            return 0
        self._fz_noise[target.data_ptr()] = target_noise
        return tsg.data_ptr()

    def _wg_plan(self, wg, grad, dev):
        """The fused weight-gradient launch plan for these members (fixed workspace pointers: built
        once, outside any graph capture): (device WgradGroup, its tile count, job table, number of
        block-assigned jobs, done counters). Job table: the fc jobs (gradient from FcFuse rows,
        final at launch start; one block each), then every other job grouped by the member tile
        range that completes its gradient -- (member, 64-row K-range) for weight tiles, the
        member's K-range-0 tiles for its bias; each such job's block (after every tile in the grid)
        waits for its range's count (UpdJob.dep = member * WG_SLOTS + slot). Noisy nets put those
        jobs first, before the fc jobs."""
        members, dims, scales = wg
        key = (tuple(tuple(m) for m in members), tuple(tuple(d) for d in dims), tuple(scales), grad.data_ptr(),
               self.wg_conv_chunks, dev)
        pl = self._wg_plans.get(key)
        if pl is None:
            assert not torch.cuda.is_current_stream_capturing(), 'fused wgrad plan: build it before capturing'
            ext = self.ext
            done = torch.zeros(32 * ext.WG_COUNTERS, dtype=torch.int32, device=dev)
            g0 = grad.data_ptr()
            lay = self.layout
            span = {}                        # tensor offset -> (member, end, is weight)
            for mi, m in enumerate(members):
                for j, ptr in enumerate(m[4:8]):           # dw, db, dw2, db2
                    if ptr:
                        o = (int(ptr) - g0) // 4
                        name = next(n for n in lay.names if lay.offsets[n] == o)
                        span[o] = (mi, o + lay.numel(name), j % 2 == 0)
            fcj, groups = [], {}
            for it in self.upd_items:
                if it[20] >= 0:
                    fcj.append(list(it))
                    continue
                src = it[1]
                owner = [(mi, w) for o, (mi, hi, w) in span.items() if o <= src < hi]
                assert len(owner) == 1, 'fused wgrad: no member writes the gradient of job at %d' % src
                mi, w = owner[0]
                if w:
                    assert it[0] == 0, 'weight gradients of fused members come as tile jobs'
                    slot = it[4] // 64                  # the tile's K-range (64 rows per fused tile)
                else:
                    slot = ext.WG_SLOTS - 1
                groups.setdefault((mi, slot), []).append(list(it))
            # range-dependent jobs right after the tiles (their waits end when the tiles do) or at the
            # end of the grid: first measured +1.2% for noisy nets, whose fc jobs run ~10 us each and
            # kept them queued to ~45 us; -0.2..-1.0% for the plain nets (profiles/r4_dep_first_ab.txt).
            # KernelTuning.dep_at = n: after the first n fc jobs; -1: noisy nets after 500 of their ~1.6k
            # fc jobs (+0.3-1.0% over 300, profiles/r5_late_ab.md), plain nets at the end
            lead = min(500, len(fcj)) if self.noisy else len(fcj)
            if self.tuning.dep_at >= 0:
                lead = max(0, min(len(fcj), int(self.tuning.dep_at)))
            table, deps = list(fcj[:lead]), []
            for (mi, slot), its in sorted(groups.items()):
                deps.append([mi, slot, len(table), len(its)])
                for it in its:                 # the job's block waits for that range's tiles
                    it[21] = mi * ext.WG_SLOTS + slot
                table += its
            table += fcj[lead:]
            host, total = ext.qnet_wgrad_plan(members, dims, scales, done, deps, conv_chunks=self.wg_conv_chunks)
            jobs = torch.tensor([v for it in table for v in it], dtype=torch.int32, device=dev)
            # (the dependent jobs: table positions [lead, lead + ndep))
            pl = (host.to(dev), int(total), jobs, len(fcj), done, lead, len(table) - len(fcj))
            self._wg_plans[key] = pl
        return pl

    def _update_split(self, opt, flat, grad, grad_scale, global_step, target, target_freq, noise, grad_noise,
                      noise_dst, next_sample, target_noise, noise_rng, fc):
        """``update_and_pack`` after ``loss_and_grad(defer_wgrad=True)``: ONE launch that also
        computes the grouped weight gradients (conv layers + output layer, fp32 atomics into
        ``grad``, optim_pack.h kModeWg). Its grid: the lead block (next minibatch + end-of-launch
        bookkeeping), the weight-gradient tiles, the fc jobs (gradient formed from the FcFuse
        rows: independent of the tiles -- the fc update, ~90% of the optimizer's bytes, runs
        beside the weight-gradient work). Every other job has a block at the end of the grid that
        waits for the tiles of its gradient's K-range."""
        from ..optim import kernel_op
        dev = flat.device
        wg, self._wg_pending = self._wg_pending, None
        fcargs = self._take_fc(fc)
        assert fcargs, 'deferred weight gradients need the fused fc gradient (defer_fc)'
        plan, nwg, jobs, nfc, _, lead, ndep = self._wg_plan(wg, grad, dev)
        # data parallelism: the dependent jobs sum their gradient over every rank inside the launch
        dp = self.dp_exchange.dpx_launch(lead, ndep) if self.dp_exchange is not None else []
        hp = opt.hp
        s0 = opt.slots[0] if len(opt.slots) > 0 else flat
        s1 = opt.slots[1] if len(opt.slots) > 1 else flat
        if getattr(opt, 'ticket', None) is None or opt.ticket.device != dev or opt.ticket.numel() < 17 * 32:
            opt.ticket = torch.zeros(17 * 32, dtype=torch.int32, device=dev)
        eff = teff = tpk = None
        if self.noisy:
            assert noise is not None and noise.dtype == torch.float32
            k = flat.data_ptr()
            p, eff = self._packed_for(k, flat), self._eff_for(k, flat)
            pt = None
            if target_noise is not None:
                assert target is not None and target_noise.dtype == torch.float32
                tk = target.data_ptr()
                tpk, teff = self._packed_for(tk, target), self._eff_for(tk, target)
        else:
            p = self.packed(flat)
            pt = self.packed(target) if target is not None else None
        hps = [float(hp['momentum']), float(hp['rho']), float(hp['rms_mom']), float(hp['rms_eps']), float(hp['b1']),
               float(hp['b2']), float(hp['adam_eps']), float(hp['ad_rho']), float(hp['ad_eps'])]
        op = kernel_op(opt)
        args = (flat, grad, s0, s1, opt.beta_powers, opt.ticket, float(opt.lr), float(opt.reg_param),
                int(opt.layout.reg_end), float(grad_scale), global_step, hps)
        self.ext.optim_pack(op, *args, jobs, p, target, pt, int(target_freq), self.opt_max_grid, noise, eff,
                            grad_noise, noise_dst,
                            (list(next_sample['spec']) + [int(next_sample['B'])]
                             if next_sample is not None and next_sample['kind'] == 'uniform' else []),
                            (list(next_sample['p']) if next_sample is not None and next_sample['kind'] == 'per' else []),
                            (list(next_sample['f']) if next_sample is not None and next_sample['kind'] == 'per' else []),
                            target_noise, teff, tpk, noise_rng, fcargs, 0, wg=plan.data_ptr(), wg_blocks=nwg,
                            dp=dp, tsg=self._tsg_arg(target, target_noise))
        if self.noisy:
            self._bound[flat.data_ptr()] = noise_dst if noise_dst is not None else noise
            if target_noise is not None:
                self._bound[target.data_ptr()] = target_noise
        return True

    def can_defer_wgrad(self, B: int, sigma_grads: bool = False) -> bool:
        """True when ``loss_and_grad(defer_fc=True, defer_wgrad=True)`` at this batch leaves the
        grouped conv / output-layer weight gradients to the next ``update_and_pack`` (which then
        runs them beside the fc update, ``_update_split``): the Nature trunk's grouped-wgrad path
        in the 16-bit builds. Under data parallelism only with ``dp_exchange`` set (the launch sums
        those gradients over the ranks itself) and the low-rank fc exchange."""
        # (the reference `cnn` too: its conv members are the same three fused tile kinds -- 8x8/4, 4x4/2,
        #  3x3/1 -- with SAME padding in their ConvArgs, conv2 / conv3 reading the pooled activations)
        return self.can_defer_fc(B, sigma_grads) and not (self.noisy and sigma_grads)

    def _take_fc(self, fc=None):
        if fc is None:
            fc, self._fc_pending = self._fc_pending, None
        if fc is None:
            return []
        x, dh, M = fc
        return [int(x), int(dh), int(M), self.FLAT, self.HH]

    def can_defer_fc(self, B: int, sigma_grads: bool = False) -> bool:
        """True when ``loss_and_grad(defer_fc=True)`` at this batch leaves the fc weight / bias
        gradient to the fused optimizer launch (16-bit builds, grouped-wgrad path)."""
        return (bool(getattr(self.ext, 'OPTIM_FC_FUSE', 0)) and self.grouped_wgrad and not self.two_stream
                and B <= 32 and not (self.noisy and sigma_grads))

    def pending_fc(self) -> bool:
        return self._fc_pending is not None or self._parts_pending is not None or self._wg_pending is not None

    def can_det_wgrad(self, B: int) -> bool:
        """True when ``loss_and_grad(det_wgrad=True)`` leaves the conv weight / bias gradients as
        deterministic chunk-group partials for the fused optimizer launch to sum (no fp32 atomics;
        the flagship Nature trunk's grouped-wgrad path)."""
        return (bool(getattr(self.ext, 'OPTIM_FC_FUSE', 0)) and self.grouped_wgrad and not self.two_stream
                and B <= 32 and self.arch.network == 'nature')

    def _det_plan(self, B: int, dev) -> dict:
        """Deterministic conv weight gradients (qnet.hip group_member partial mode): member i's
        M rows split into 128-row chunks, ``mloop`` consecutive chunks per chunk group summed in
        registers in a fixed order, each group's [K][N] weights + [N] bias stored plainly into
        its own partial slice; the optimizer's conv jobs then sum the slices in ascending order.
        Same result on every run (and every rank) for the same inputs. At most 26 partial slices
        per layer (the round-3 sweep's best: fewer slices sum fewer bytes but lengthen the wgrad
        blocks, profiles/r3_det_wgrad.md)."""
        key = (B, dev.index if dev.index is not None else 0)
        pl = self._det.get(key)
        if pl is not None:
            return pl
        lay = self.layout
        cap = 26
        info, base = {}, 0
        for c in self.arch.convs:
            h, w = c.conv_hw
            K, N = c.k * c.k * c.cin, c.cout
            nch = (B * h * w + 127) // 128
            mloop = (nch + cap - 1) // cap
            ng = (nch + mloop - 1) // mloop
            stride = (K * N + N + 63) // 64 * 64
            info[c.name] = (base, K, N, ng, stride, mloop)
            base += ng * stride
        buf = torch.zeros(base, dtype=torch.float32, device=dev)
        by_off = {}
        for name, (b0, K, N, ng, stride, _) in info.items():
            by_off[lay.offsets[name + '/w']] = (b0, ng, stride)
            by_off[lay.offsets[name + '/b']] = (b0 + K * N, ng, stride)
        first, rest = [], []
        for it in self.upd_items:
            it = list(it)
            # tile jobs: src_off is the tensor's; chunk jobs: the chunk's (bias chunks start at 0)
            hit = by_off.get(it[1])
            if hit is not None:
                it[-3:] = list(hit)
                first.append(it)     # the long-latency summing jobs first in the launch
            else:
                rest.append(it)
        ints = [v for it in first + rest for v in it]
        pl = {'buf': buf, 'info': info,
              'jobs': torch.tensor(ints, dtype=torch.int32, device=dev)}
        self._det[key] = pl
        return pl

    def _det_member(self, pl, name):
        b0, _, _, _, stride, mloop = pl['info'][name]
        return [pl['buf'].data_ptr() + 4 * b0, stride, mloop]

    def _plan_noisy(self):
        """Mix jobs (rainbow.hip NoisyJob): every mu tensor -> the effective buffer;
        noisy dense layers add sigma * f(eps_in) f(eps_out). Noise offsets follow
        models/torch_net.forward (dense layers in arch.dense_layers() order)."""
        self.noisy_jobs = []
        if not self.noisy:
            return
        lay = self.layout
        noff, dense = 0, {}
        for d in self.arch.dense_layers():
            if d.noisy:
                dense[d.name] = (d, noff)
                noff += d.fin + d.fout
        # (eps_in, eps_out) offsets of the fc layer(s) in fc/fwd column order (factorised forward)
        fcn = ['value/fcl', 'advantage/fcl'] if self.dueling else ['fcl', 'fcl']
        if all(n in dense for n in fcn):
            self._fz_offs = [(dense[n][1], dense[n][1] + dense[n][0].fin) for n in fcn]
        elif self.tfact:
            self.tfact = False
        for name in lay.names:
            kind = lay.kinds[name]
            if kind not in ('w', 'b'):
                continue
            layer = name.rsplit('/', 1)[0]
            n = lay.numel(name)
            if layer in dense:
                d, o = dense[layer]
                if kind == 'w':
                    self.noisy_jobs.append([lay.offsets[name], lay.offsets[layer + '/w_sigma'], d.fin, d.fout, o,
                                            o + d.fin, 0, 0])
                else:
                    self.noisy_jobs.append([lay.offsets[name], lay.offsets[layer + '/b_sigma'], 1, d.fout, -1,
                                            o + d.fin, 0, 0])
            else:
                self.noisy_jobs.append([lay.offsets[name], -1, 1, n, -1, -1, 0, 0])
        self._noisy_max = max(j[2] * j[3] for j in self.noisy_jobs)
        self._noisy_dev: Dict[torch.device, torch.Tensor] = {}

    def _noisy_jobs_on(self, dev):
        t = self._noisy_dev.get(dev)
        if t is None:
            ints = [v for j in self.noisy_jobs for v in j]
            assert len(ints) == len(self.noisy_jobs) * self.ext.NOISY_JOB_INTS
            t = torch.tensor(ints, dtype=torch.int32, device=dev)
            self._noisy_dev[dev] = t
        return t

    def effective(self, flat: torch.Tensor, noise: Optional[torch.Tensor], key: Optional[int] = None
                  ) -> torch.Tensor:
        """Noisy nets: eff = mu + sigma*f(e_in)f(e_out) for the noisy layers (mu elsewhere),
        packed into ``flat``'s fragment buffer (or ``key``'s) in one launch. Returns the
        effective fp32 buffer the kernels read biases / head weights from. No launch when
        ``noise`` is bound to ``flat`` (``premix``); no-op (returns flat) without noisy layers."""
        if not self.noisy:
            return flat
        k = flat.data_ptr() if key is None else key
        if key is None and noise is not None and self._bound.get(k) is noise:
            return self._eff[k]
        if key is None:
            self._bound.pop(k, None)
        eff = self._eff_for(k, flat)
        p = self._packed_for(k, flat)
        self._mix_pack(flat, noise, eff, p)
        return eff

    def _packed_for(self, key: int, like: torch.Tensor) -> torch.Tensor:
        p = self._packed.get(key)
        if p is None:
            p = torch.zeros(self.packed_elems, dtype=self.act_dtype, device=like.device)
            self._packed[key] = p
        return p

    def _jobs_on(self, dev):
        t = self._jobs_dev.get(dev)
        if t is None:
            ints = [v for j in self.jobs for v in j.ints()]
            assert len(ints) == len(self.jobs) * self.ext.PACK_JOB_INTS
            t = torch.tensor(ints, dtype=torch.int32, device=dev)
            self._jobs_dev[dev] = t
        return t

    def packed(self, flat: torch.Tensor) -> torch.Tensor:
        key = flat.data_ptr()
        p = self._packed.get(key)
        if p is None:
            p = torch.zeros(self.packed_elems, dtype=self.act_dtype, device=flat.device)
            self._packed[key] = p
            self.repack(flat)
        return p

    def repack(self, flat: torch.Tensor, target: Optional[torch.Tensor] = None,
               step: Optional[torch.Tensor] = None, freq: int = 1):
        """fp32 master -> bf16 MFMA fragments (call after every optimizer step / load).

        target/step/freq: also write the fragments into ``target``'s packed copy when
        step % freq == 0 (device predicate; the fused hard target sync)."""
        bound = self._bound.get(flat.data_ptr()) if self.noisy else None
        if bound is not None:                    # noisy: keep the bound noise sample mixed in
            self.premix(flat, bound)
            return
        p = self._packed.get(flat.data_ptr())
        if p is None:
            self.packed(flat)
            if target is None:
                return
            p = self._packed[flat.data_ptr()]
        jobs = self._jobs_on(flat.device)
        if target is not None:
            assert step is not None and step.dtype == torch.int64 and step.device == flat.device
            pt = self.packed(target)
            self.ext.qnet_pack(flat.data_ptr(), p.data_ptr(), jobs.data_ptr(), len(self.jobs), self._max_threads,
                               pt.data_ptr(), step.data_ptr(), int(freq))
            return
        self.ext.qnet_pack(flat.data_ptr(), p.data_ptr(), jobs.data_ptr(), len(self.jobs), self._max_threads)

    def sync_target(self, target: torch.Tensor, online: torch.Tensor, tau: float,
                    step: Optional[torch.Tensor] = None, freq: int = 1):
        """Refresh the target's packed copy after a target update of the fp32 master."""
        from . import kernels
        bound = self._bound.get(target.data_ptr()) if self.noisy else None
        if bound is not None:               # noisy: re-mix the (possibly) new target under its noise
            self.premix(target, bound)
            return
        pt = self.packed(target)
        if tau >= 1.0:
            po = self.packed(online)
            # bit-identical to repacking the copied fp32 weights; same device predicate
            kernels.target_update(pt.view(torch.float32), po.view(torch.float32), 1.0, step, freq)
        else:
            self.repack(target)

    # ------------------------------------------------------------ streams
    def lowrank_spec(self, B: int, sigma_fused: bool = False, fused_fc: bool = False):
        """Low-rank DP exchange of the fc (hidden dense) layer's weight gradient, when this
        executor's grouped-wgrad Nature path runs at this batch: dW = X^T dH has rank <= B, so
        instead of all-reducing dW (1.6M values per hidden layer) the ranks all-gather X (the fc
        input rows, B x F) and dH (B x HH) and every rank forms the summed dW over all W*B rows
        itself -- bit-identical on every rank (one fixed-order, atomic-free launch). Returns
        {'ranges': [(lo, hi), ...] of the fc weight tensors in the flat buffer (the caller
        all-reduces the complement), 'skip': ranges whose gradient is never read (noisy nets with
        ``sigma_fused``: the sigma tensors, whose gradient the fused optimizer derives from the
        all-reduced mu gradient), 'gather_bytes': per-rank payload} or None. Noisy nets: the
        factors are those of dL/dW_eff, which IS the mu gradient. ``fused_fc``: the optimizer launch
        forms dW (and the fc bias gradient) from the gathered rows itself, so the fc biases leave
        the all-reduce as well ('skip')."""
        if (self.arch.network != 'nature' or (self.noisy and not sigma_fused) or not self.grouped_wgrad
                or self.two_stream or B > 32):
            return None
        lay = self.layout
        names = ['value/fcl/w', 'advantage/fcl/w'] if self.dueling else ['fcl/w']
        if not all(n in lay.offsets for n in names):
            return None
        skip = [(lay.offsets[n], lay.offsets[n] + lay.numel(n)) for n in lay.names
                if self.noisy and (n.endswith('/w_sigma') or n.endswith('/b_sigma'))]
        if fused_fc:
            skip += [(lay.offsets[n[:-2] + '/b'], lay.offsets[n[:-2] + '/b'] + lay.numel(n[:-2] + '/b')) for n in names]
        return {'ranges': [(lay.offsets[n], lay.offsets[n] + lay.numel(n)) for n in names], 'skip': skip,
                'gather_bytes': B * (self.FLAT + self.HH) * self.esz}

    def _lowrank_ws(self, B: int, W: int, dev) -> dict:
        key = (B, W, dev)
        lw = getattr(self, '_lr_bufs', {}).get(key)
        if lw is None:
            if not hasattr(self, '_lr_bufs'):
                self._lr_bufs = {}
            lw = {'x': torch.zeros(W * B * self.FLAT, dtype=self.act_dtype, device=dev),
                  'dh': torch.zeros(W * B * self.HH, dtype=self.act_dtype, device=dev)}
            self._lr_bufs[key] = lw
        return lw

    def _side_stream(self, dev):
        st = getattr(self, '_side', None)
        if st is None or st.device != dev:
            st = torch.cuda.Stream(device=dev)
            self._side = st
            self._events = {}
        return st

    def _event(self, name, stream):
        ev = self._events.get(name)
        if ev is None:
            ev = torch.cuda.Event()
            self._events[name] = ev
        ev.record(stream)
        return ev

    # ---------------------------------------------------------- workspace
    def _workspace(self, B: int, dev) -> dict:
        key = (B, dev.index if dev.index is not None else 0)
        ws = self._ws.get(key)
        if ws is not None:
            return ws
        bf = dict(dtype=self.act_dtype, device=dev)
        c1, c2, c3 = self.arch.convs
        h1, w1 = c1.out_hw
        h2, w2 = c2.out_hw
        h3, w3 = c3.out_hw
        ws = {
            'x1': torch.zeros(3, B * h1 * w1 * c1.cout, **bf),
            'x2': torch.zeros(3, B * h2 * w2 * c2.cout, **bf),
            'x3': torch.zeros(4, B * h3 * w3 * c3.cout, **bf),     # 4th row: fused-acting instance
            'h': torch.zeros(4, B * self.HH, **bf),
            'dh': torch.zeros(B * self.HH, **bf),
            'dz3': torch.zeros(B * self.FLAT, **bf),
            'dz2': torch.zeros(B * h2 * w2 * c2.cout, **bf),
            'dz1': torch.zeros(B * h1 * w1 * c1.cout, **bf),
            'loss': torch.zeros(1, dtype=torch.float32, device=dev),
            'prio': torch.zeros(B, dtype=torch.float32, device=dev),
            'q': torch.zeros(B * self.A, dtype=torch.float32, device=dev),
            'ones': torch.ones(B, dtype=torch.float32, device=dev),
        }
        ws.update(self._head_ws(B, dev))
        self._ws[key] = ws
        return ws

    def _head_ws(self, B, dev) -> dict:
        """Per-block loss partials of the head launch (summed by the fc dgrad launch) and the
        head's dZ rows as act_t: scalar heads dQ [B][64]; C51 dL/dlogits [B][KD] (the dH igemm's
        A operand; its pad columns stay zero from here on)."""
        f32 = dict(dtype=torch.float32, device=dev)
        width = self.c51_KD if self.dist else 64
        return {'loss_parts': torch.zeros(64, **f32), 'dq16': torch.zeros(B * width, dtype=self.act_dtype, device=dev)}

    def _loss_parts(self, B):
        """Loss partials the head launch writes: one per 16-sample tile (scalar) or per C51
        learner block (8 samples each, at most 64 blocks)."""
        return min((B + 7) // 8, 64) if self.dist else (B + 15) // 16

    # ------------------------------------------------------------ forward
    @property
    def fused_sampling(self) -> bool:
        """The fused trunk can draw the uniform minibatch itself (replay.sample_slots(defer))."""
        return self.fused_trunk

    def _fwd_trunk(self, xs, packs, flats, ws, B, ninst, frames=None, keep_acts=True, M=(), sample=None, fc=True):
        """conv1..fc for `ninst` instances -> ws['h'] (M: valid rows per instance, e.g. the
        fused actor instance's E < B). sample: (spec pointers, sampled instances) — the
        trunk draws the uniform batch itself (the slot tables of those instances are outputs).
        fc=False: stop at conv3 (the caller's fused fc + head launch follows, ``_fc_head``).

        xs: uint8 NHWC [B, 84, 84, 4] inputs, or (frames given) int32 [B, 4] slot
        tables into the frame ring ``frames`` [F, 84, 84] (fused gather)."""
        ext, lay = self.ext, self.layout
        c1, c2, c3 = self.arch.convs
        (h1, w1), (h2, w2), (h3, w3) = c1.out_hw, c2.out_hw, c3.out_hw
        bias = lambda name: [f.data_ptr() + 4 * lay.offsets[name] for f in flats]
        pk = lambda key: [p.data_ptr() + self.esz * self.poff[key] for p in packs]
        rows = lambda t, i: t[i].data_ptr()
        if self.fused_trunk:
            # ONE launch for conv1..conv3: a workgroup per (sample, instance), activations in LDS
            pad = lambda v: list(v) + [0] * (4 - len(v))
            slots = [x.data_ptr() for x in xs] if frames is not None else []
            states = [] if frames is not None else [x.data_ptr() for x in xs]
            ptrs = (pad(slots) + pad(states) + pad(pk('conv1/fwd')) + pad(pk('conv2/fwd')) + pad(pk('conv3/fwd'))
                    + pad(bias('conv1/b')) + pad(bias('conv2/b')) + pad(bias('conv3/b'))
                    # only the online(s) instance feeds the backward: the others skip x1/x2
                    + pad([rows(ws['x1'], 0)] if keep_acts else []) + pad([rows(ws['x2'], 0)] if keep_acts else [])
                    + pad([rows(ws['x3'], i) for i in range(ninst)]))
            prof = self.trunk_prof.data_ptr() if self.trunk_prof is not None else 0
            smp = list(sample[0]) + [int(sample[1])] if sample is not None else []
            ext.qnet_trunk(frames.data_ptr() if frames is not None else 0, ptrs, B, ninst, self.input_scale, prof,
                           list(M), smp)
            if fc:
                self._fc_fwd(packs, flats, ws, B, ninst)
            return
        d1 = [B * h1 * w1, c1.cout, c1.k * c1.k * c1.cin, (c1.cout + 15) // 16, c1.cout, 84, 84, h1, w1, 0, 0]
        kind1 = _KIND['C1']
        if frames is not None:
            d1 += [frames.data_ptr(), 84 * 84]
            kind1 = _KIND['F1']
        ext.qnet_igemm(kind1, [x.data_ptr() for x in xs], pk('conv1/fwd'), bias('conv1/b'),
                       [rows(ws['x1'], i) for i in range(ninst)], [], [self.input_scale] * ninst, d1)
        ext.qnet_igemm(_KIND['C2'], [rows(ws['x1'], i) for i in range(ninst)], pk('conv2/fwd'), bias('conv2/b'),
                       [rows(ws['x2'], i) for i in range(ninst)], [], [1.0] * ninst,
                       [B * h2 * w2, c2.cout, c2.k * c2.k * c2.cin, c2.cout // 16, c2.cout, h1, w1, h2, w2, 0, 0])
        ext.qnet_igemm(_KIND['C3'], [rows(ws['x2'], i) for i in range(ninst)], pk('conv3/fwd'), bias('conv3/b'),
                       [rows(ws['x3'], i) for i in range(ninst)], [], [1.0] * ninst,
                       [B * h3 * w3, c3.cout, c3.k * c3.k * c3.cin, c3.cout // 16, c3.cout, h2, w2, h3, w3, 0, 0])
        if fc:
            self._fc_fwd(packs, flats, ws, B, ninst)

    def _fc_fwd(self, packs, flats, ws, B, ninst):
        fcb = [p.data_ptr() + self.esz * self.poff['fc/bias'] for p in packs]
        z = self._fc_zero                  # (the step's dgrad-chain counters: zeroed by this launch)
        self.ext.qnet_igemm(_KIND['DFWD'], [ws['x3'][i].data_ptr() for i in range(ninst)],
                            [p.data_ptr() + self.esz * self.poff['fc/fwd'] for p in packs], fcb,
                            [ws['h'][i].data_ptr() for i in range(ninst)], [], [1.0] * ninst,
                            [B, self.HH, self.FLAT, self.HH // 16, self.HH, 0, 0, 0, 0, 0, 0],
                            [z.data_ptr(), z.numel(), 0, 0, 0] if z is not None else [], [1.0] if z is not None else [],
                            fz=self._fz_args(packs[:ninst], B))

    def _fz_args(self, packs, B) -> list:
        """The fc forward's factorised instance (``set_factorised``): [inst, sigma fragments, noise,
        nsplit, eps_in / eps_out offsets of both column halves], or [] when no instance is."""
        if not self._fact_pk:
            return []
        idx = [i for i, p in enumerate(packs) if p.data_ptr() in self._fact_pk]
        if not idx:
            return []
        assert len(idx) == 1 and B <= 32, 'factorised fc forward: one instance, B <= 32'
        k = self._fact_pk[packs[idx[0]].data_ptr()]
        noise = self._fz_noise.get(k)
        assert noise is not None, 'factorised target: not mixed yet (premix / effective first)'
        (e0, o0), (e1, o1) = self._fz_offs
        return [idx[0], self._fact[k].data_ptr() + self.esz * self.poff['fc/fwd'], noise.data_ptr(),
                self.HID if self.dueling else self.HH, e0, o0, e1, o1]

    def can_fold_head(self, B: int, E: int = 0) -> bool:
        """Whether the training step's fc forward and scalar head run as ONE launch
        (csrc/kernels/fc_head.hip): scalar heads with A <= 18, hidden width <= 512, <= 16 fused
        actors, a hidden width % 64 == 0."""
        return (self.fold_head and not self.dist and self.A <= 18 and self.HID <= 512 and self.HID % 64 == 0
                and E <= 16 and B <= 1024)

    def _fold_ws(self, B, dev) -> dict:
        key = ('fold', B, dev.index if dev.index is not None else 0)
        ws = self._ws.get(key)
        if ws is None:
            mpad = (B + 15) // 16 * 16
            ws = {'q': torch.zeros(4 * mpad * 32 * (self.HH // 16), dtype=torch.float32, device=dev),
                  'cnt': torch.zeros(mpad // 16 + 2, dtype=torch.int32, device=dev), 'mpad': mpad,
                  'dqg': torch.zeros(mpad * 32, dtype=torch.float32, device=dev),
                  'epoch': torch.zeros(mpad // 16 + 2, dtype=torch.int32, device=dev)}
            self._ws[key] = ws
        return ws

    def fold_errors(self) -> list:
        """Error words of the folded head launches (host sync): 0x1000000 | group for a dH-tile
        block whose wait for its group's dQ expired (fc_head.hip; the block skipped its dH write).
        The word is the epoch buffer's last entry (ngroups + 1) and is never cleared."""
        out = []
        for key, ws in self._ws.items():
            if isinstance(key, tuple) and key and key[0] == 'fold':
                v = int(ws['epoch'][ws['mpad'] // 16 + 1].item())
                if v:
                    out.append(v)
        return out

    def _fc_head(self, packs, ws, B, nlearn, ints, w, b, wv, bv, io, actor, actor_f, act_h, dev):
        """fc forward of every instance (learners', then the fused actors') + the scalar head's
        loss / dQ / dH (+ the fused acting step) in ONE launch (``can_fold_head``)."""
        n = len(packs)
        fw = self._fold_ws(B, dev)
        self.ext.qnet_fc_head([ws['x3'][i].data_ptr() for i in range(n)],
                              [p.data_ptr() + self.esz * self.poff['fc/fwd'] for p in packs],
                              [p.data_ptr() + self.esz * self.poff['fc/bias'] for p in packs],
                              [ws['h'][i].data_ptr() for i in range(n)],
                              [B, self.HH, self.FLAT, self.HH // 16, self.HH, 0, 0, 0, 0, 0, 0],
                              ints, [self.delta], [ws['h'][i].data_ptr() for i in range(nlearn)], w, b, wv, bv, io,
                              [ws['loss_parts'].data_ptr(), ws['dq16'].data_ptr()], actor, actor_f, act_h,
                              [fw['q'].data_ptr(), fw['cnt'].data_ptr(), fw['mpad'], nlearn,
                               fw['dqg'].data_ptr() if self.fold_spin else 0, fw['epoch'].data_ptr()] +
                              ([self._fc_zero.data_ptr(), self._fc_zero.numel()] if self._fc_zero is not None else []),
                              self.fold_prof.data_ptr() if self.fold_prof is not None else 0,
                              two_per_cu=bool(self.tuning.fold_two_per_cu))

    def _head_ptrs(self, flats):
        lay = self.layout
        off = lambda f, n: f.data_ptr() + 4 * lay.offsets[n]
        if self.dueling:
            w = [off(f, 'advantage/output/w') for f in flats]
            b = [off(f, 'advantage/output/b') for f in flats]
            wv = [off(f, 'value/output/w') for f in flats]
            bv = [off(f, 'value/output/b') for f in flats]
        else:
            w = [off(f, 'output/w') for f in flats]
            b = [off(f, 'output/b') for f in flats]
            wv, bv = [], []
        return w, b, wv, bv

    def _check_states(self, x):
        assert x.dtype == torch.uint8 and x.is_contiguous() and tuple(x.shape[1:]) == (84, 84, 4), \
            'HIP executor expects uint8 NHWC [B, 84, 84, 4] states, got %s %s' % (x.dtype, tuple(x.shape))

    def forward(self, flat, x, noise=None):
        return self.q_values(flat, x, noise)

    def _c51_logits(self, hs, pwc, pbias):
        """C51 logits of every instance as fp32 rows [B][KD] (logits | pad | dueling value logits
        at VO) from ONE igemm launch over the combined output layer (``head/wc``): spread over
        many CUs instead of re-streaming the output layer through one CU per head workgroup."""
        B, KD = self._c51_B, self.c51_KD
        n = len(hs)
        ws = self._c51_ws(B)
        lg = [ws['lg'][i].data_ptr() for i in range(n)]
        self.ext.qnet_igemm(_KIND['DF32'], list(hs), pwc, pbias, lg, [], [1.0] * n,
                            [B, KD, self.HH, KD // 16, KD, 0, self.HH, 0, 0, 0, 0])
        return lg

    def _c51_ws(self, B):
        key = ('c51', B)
        ws = self._ws.get(key)
        if ws is None:
            ws = {'lg': torch.zeros(4, B * self.c51_KD, dtype=torch.float32, device=self._c51_dev)}
            self._ws[key] = ws
        return ws

    def _head(self, ints, hs, w, b, wv, bv, io, pw, pwv, zero, actor, actor_f, act_h=0, ws=None):
        """Output layer + loss (+ backward) launch: scalar head or the C51 head."""
        if self.dist:
            self._c51_B = ints[0]
            # (pw, pwv = the combined output layer's fragments and bias rows, see _head_packs)
            if act_h:
                # fused acting: the actors' logits ride in the same igemm launch as one more
                # instance (online weights), the acting step in more C51-head workgroups
                lg = self._c51_logits(list(hs) + [act_h], list(pw) + [pw[0]], list(pwv) + [pwv[0]])
            else:
                lg = self._c51_logits(hs, pw, pwv)
            qp = [ws['loss_parts'].data_ptr(), ws['dq16'].data_ptr()] if not ints[5] else []
            prof = self.head_prof.data_ptr() if self.head_prof is not None and not ints[5] else 0
            self.ext.qnet_c51_head(ints, [self.atoms], [float(self.arch.v_min), float(self.arch.v_max)], hs, w, b,
                                   wv, bv, io, [], [], zero, actor, actor_f, prof, lg, act_h, qp)
        else:
            prof = self.head_prof.data_ptr() if self.head_prof is not None else 0
            self.ext.qnet_head_loss(ints, [self.delta], hs, w, b, wv, bv, io, pw, pwv,
                                    [ws['loss_parts'].data_ptr(), ws['dq16'].data_ptr()], actor, actor_f, act_h, prof)

    def q_values(self, flat: torch.Tensor, x: torch.Tensor, noise=None) -> torch.Tensor:
        """Q [B, A] (C51: expected value of the return distribution)."""
        x = x.contiguous()
        self._check_states(x)
        B = x.shape[0]
        ws = self._workspace(B, x.device)
        fl = self.effective(flat, noise)
        p = self.packed(flat)
        self._fwd_trunk([x], [p], [fl], ws, B, 1, keep_acts=False)
        w, b, wv, bv = self._head_ptrs([fl])
        q = torch.empty(B, self.A, dtype=torch.float32, device=x.device)
        pw, pwv = self._head_packs([p])
        self._c51_dev = x.device
        self._head([B, self.A, self.HID, int(self.dueling), 0, 1], [ws['h'][0].data_ptr()],
                   w, b, wv, bv, [0] * 7 + [q.data_ptr()] + [0] * 5, pw, pwv, [], [], [], ws=ws)
        return q

    def act_fused(self, flat: torch.Tensor, frames: torch.Tensor, stacks: torch.Tensor, actor_ptrs, actor_ints,
                  actor_f, q_out: Optional[torch.Tensor] = None, noise: Optional[torch.Tensor] = None):
        """Acting step in 3 launches: fused trunk (frame ring via the actors' slot stacks)
        -> fc -> head with the eps-greedy/env/replay-append step fused (+2 for noisy nets:
        parameter mix and repack under the acting noise)."""
        E = stacks.shape[0]
        assert stacks.dtype == torch.int32 and stacks.is_contiguous() and stacks.shape[1] == 4
        ws = self._workspace(E, frames.device)
        fl = self.effective(flat, noise)
        p = self.packed(flat)
        self._fwd_trunk([stacks], [p], [fl], ws, E, 1, frames=frames, keep_acts=False)
        w, b, wv, bv = self._head_ptrs([fl])
        pw, pwv = self._head_packs([p])
        self._c51_dev = frames.device
        self._head([E, self.A, self.HID, int(self.dueling), 0, 1], [ws['h'][0].data_ptr()],
                   w, b, wv, bv, [0] * 7 + [q_out.data_ptr() if q_out is not None else 0] + [0] * 5,
                   pw, pwv, [], list(actor_ptrs) + list(actor_ints), list(actor_f), ws=ws)

    def _head_packs(self, packs):
        """Scalar heads: the output layer's fragments (plain / advantage, dueling value); C51: the
        combined output layer's fragments and its fp32 bias row."""
        if self.dist:
            return ([p.data_ptr() + self.esz * self.poff['head/wc'] for p in packs],
                    [p.data_ptr() + self.esz * self.poff['head/bias'] for p in packs])
        pw = [p.data_ptr() + self.esz * self.poff['head/w'] for p in packs]
        pwv = [p.data_ptr() + self.esz * self.poff['head/v'] for p in packs] if self.dueling else []
        return pw, pwv

    def _c51_dh(self, ws, B, po):
        """C51: dH = (dout16 [W | Wv]^T) * (h > 0) on the igemm kernel (packed dgrad fragments)."""
        HH = self.HH
        self.ext.qnet_igemm(_KIND['DDGRAD'], [ws['dq16'].data_ptr()],
                            [po.data_ptr() + self.esz * self.poff['head/dgrad']], [], [ws['dh'].data_ptr()],
                            [ws['h'][0].data_ptr()], [1.0], [B, HH, self.c51_KD, HH // 16, HH, 0, 0, 0, 0, 0, 0])

    def _fc_dgrad(self, ws, B, po, zero=(), draw_noise=None, dh_done=False, gather=None):
        """dz3 = (dH W_fc^T) * (x3 > 0) on the igemm kernel; the launch also zeroes the conv
        weight-gradient range and sums the head's loss partials (side duties). Scalar heads: the
        head kernel wrote dH; C51: dH = (dout16 [W | Wv]^T) * (h > 0) is one more igemm launch
        before it, over the head's dL/dlogits rows. draw_noise = (out0, out1, rng): the launch
        also draws the next noisy-net samples (see ``loss_and_grad``)."""
        if self.dist and not dh_done:
            self._c51_dh(ws, B, po)
        dh, pk, dz3, x3, dims, aux, aux_f = self._fc_dgrad_args(ws, B, po, zero, draw_noise)
        if gather is not None:          # (device XgmiGatherArgs ptr, blocks): the low-rank all-gather duty
            aux += [int(gather[0]), int(gather[1])]
        self.ext.qnet_igemm(_KIND['DDGRAD'], [dh], [pk], [], [dz3], [x3], [1.0], dims, aux, aux_f)

    def _fc_dgrad_args(self, ws, B, po, zero=(), draw_noise=None):
        """(dH, packed W_fc dgrad fragments, dz3, x3 mask, dims, aux, aux_f) of the fc dgrad launch:
        aux = the side duties (zero the conv gradient range, sum the loss partials, draw noise)."""
        F, HH = self.FLAT, self.HH
        pk = po.data_ptr() + self.esz * self.poff['fc/dgrad']
        zp, zn = (zero[0], zero[1]) if zero else (0, 0)
        aux = [zp, zn, ws['loss_parts'].data_ptr(), self._loss_parts(B), ws['loss'].data_ptr()]
        if draw_noise is not None:
            o0, o1, rng = draw_noise
            assert o0.dtype == torch.float32 and (o1 is None or o1.numel() == o0.numel()) and rng.dtype == torch.int64
            aux += [o0.data_ptr(), o1.data_ptr() if o1 is not None else 0, o0.numel(), rng.data_ptr()]
        return (ws['dh'].data_ptr(), pk, ws['dz3'].data_ptr(), ws['x3'][0].data_ptr(),
                [B, F, HH, F // 16, F, 0, 0, 0, 0, 0, 0], aux, [1.0 / B])

    def can_chain_dgrad(self, B: int) -> bool:
        """Whether the Nature backward's fc / conv3 / conv2 dgrads run as ONE launch
        (qnet.hip dgrad_chain_kernel): 16-bit or fp32 builds, the grouped-wgrad path, one stream."""
        return (self.chain_dgrad and self.arch.network == 'nature' and self.grouped_wgrad and not self.two_stream
                and B <= 1024 and self.FLAT % 64 == 0 and self.arch.convs[2].cin == 64)

    def chain_error(self, B, dev) -> bool:
        """True if a dgrad-chain stage gave up waiting for its inputs (host sync)."""
        return int(self._chain_ws(B, dev)[((B + 15) // 16 + B) * 32]) != 0

    def _chain_ws(self, B, dev):
        key = ('chain', B, dev.index if dev.index is not None else 0)
        t = self._ws.get(key)
        if t is None:
            n = ((B + 15) // 16 + B + 1) * 32         # one counter per 128-byte line
            t = torch.zeros(n, dtype=torch.int32, device=dev)
            self._ws[key] = t
        return t

    def _head_wgrad_members(self, ws, B, h0, hgrads):
        """Grouped-wgrad members of the output layer: dW = h^T dZ (dueling: advantage stream over
        h's second half, value stream over its first half) from the head's dZ rows (dq16):
        scalar heads dQ (ld 64, value dQ in column 32), C51 dL/dlogits (ld KD, value at VO)."""
        dw, db, dwv, dbv = hgrads
        H, HH = self.HID, self.HH
        N, NV = (self.NO, self.atoms) if self.dist else (self.A, 1)
        ld, vo = (self.c51_KD, self.c51_VO) if self.dist else (64, 32)
        dq = ws['dq16'].data_ptr()
        esz = ws['dq16'].element_size()
        if not self.dueling:
            return ([[_KIND['HW'], h0, dq, ld, dw, db, 0, 0, N, N]], [[B, N, H, 0, 0, 0, HH, 0, 0, 0, 0]])
        return ([[_KIND['HW'], h0 + esz * H, dq, ld, dw, db, 0, 0, N, N],
                 [_KIND['HW'], h0, dq + esz * vo, ld, dwv, dbv, 0, 0, NV, NV]],
                [[B, N, H, 0, 0, 0, HH, 0, 0, 0, 0], [B, NV, H, 0, 0, 0, HH, 0, 0, 0, 0]])

    # ----------------------------------------------------------- training
    def supports_fused_acting(self) -> bool:
        return not self.two_stream

    def loss_and_grad(self, online: torch.Tensor, target: torch.Tensor, batch: Dict[str, torch.Tensor],
                      grad_out: torch.Tensor, noise=None, noise_target=None, acting: Optional[dict] = None,
                      split: bool = False, sigma_grads: bool = True, draw_noise=None, lowrank=None,
                      defer_fc: bool = False, det_wgrad: bool = False, defer_wgrad: bool = False):
        """lowrank (data parallelism, see ``lowrank_spec``): {'gather': f(srcs, outs, nbytes) (an
        in-stream all-gather of two byte segments), 'world', 'rank'}. With ``split``, the fc weight
        gradient is then formed from the all-gathered factors right after the head, in stream order
        (ranks != 0 store zeros into the fc bias gradient, so the caller's all-reduce of the
        remaining range sums it exactly once).

        defer_fc (``can_defer_fc``): the fc weight and bias gradients are NOT written to grad_out;
        the next ``update_and_pack`` forms them from the fc input rows and dH rows (this rank's, or
        the all-gathered ones under ``lowrank``) inside the optimizer launch.

        defer_wgrad (``can_defer_wgrad``, with defer_fc, one process): the grouped conv and
        output-layer weight / bias gradients are NOT launched here either; the next
        ``update_and_pack`` computes them in the leading blocks of its first launch, beside the fc
        update (``_update_split``). ``grad_out`` holds them only after that call.

        det_wgrad (``can_det_wgrad``, one process): the conv weight / bias gradients are NOT
        written to grad_out either; the grouped wgrad launch stores per-chunk-group partials
        (``_det_plan``) and the next ``update_and_pack`` sums them in a fixed order: no fp32
        atomics, no zeroing of the conv range, bit-reproducible.

        sigma_grads=False (noisy nets): leave the sigma slots of grad_out alone — the fused
        optimizer derives dL/dsigma from the mu-slot gradient and the noise itself.

        draw_noise = (out0, out1, rng) (noisy nets, fused optimizer to follow): the fc dgrad launch
        also draws the next noise samples from the device stream ``rng`` into out0 / out1 (no
        launch of its own); ``update_and_pack(noise_rng=rng)`` then advances the stream.

        acting (fused acting, slot batches only): {'stacks': [E, 4] int32 frame slots of the
        device actors' states, 'ptrs', 'ints', 'f': the actor-step arguments of act_fused}. The
        actors' states ride along as one more trunk / fc instance with the online weights, and
        one extra workgroup of the head launch runs the eps-greedy / env / replay-append step:
        acting costs no launches of its own. (The learner's minibatch is drawn before this
        step's transitions land: a one-step lag vs acting first.)

        split (data parallelism): return ``(loss, prio, tail)`` where this call has launched
        everything up to the dense-layer weight gradients (the dense range of the flat gradient,
        ~95% of Nature-CNN's bytes, is final when it returns) and ``tail()`` launches the conv
        backward. The learner starts the all-reduce of the dense range between the two, so it
        overlaps the conv backward. ``tail`` is None when this network has no split point."""
        ext, lay = self.ext, self.layout
        gnoise = noise if sigma_grads else None      # noise of the dL/dsigma split (None: skip it)
        frames = batch.get('frames')
        if frames is not None:             # slot batch: conv1 reads the replay frame ring directly
            s, ns = batch['state_slots'], batch['next_slots']
            assert s.dtype == torch.int32 and s.shape[1] == 4 and s.is_contiguous() and ns.is_contiguous()
            assert frames.dtype == torch.uint8 and tuple(frames.shape[1:]) == (84, 84)
        else:
            s, ns = batch['states'], batch['next_states']
            self._check_states(s)
            self._check_states(ns)
        B = s.shape[0]
        assert B <= 1024
        dev = s.device
        ws = self._workspace(B, dev)
        po, pt = self.packed(online), self.packed(target)
        # noisy nets: effective weights under this step's noise (mixed + packed on the GPU)
        eo, et = self.effective(online, noise), self.effective(target, noise_target)
        ninst = 3 if self.double else 2
        xs = [s, ns, ns][:ninst]
        packs = [po, pt, po][:ninst]
        flats = [eo, et, eo][:ninst]
        if acting is not None:
            assert frames is not None and self.supports_fused_acting(), 'fused acting needs a slot batch'
            E = acting['stacks'].shape[0]
            assert acting['stacks'].dtype == torch.int32 and acting['stacks'].is_contiguous() and E <= B
        # conv weight/bias grads are accumulated with atomics across M-chunks: the head
        # kernel zeroes that range in-kernel; fc grads are plain stores while B <= 32
        conv_lo = lay.offsets[self.arch.convs[0].name + '/w']
        conv_hi = max(lay.offsets[c.name + '/b'] + c.cout for c in self.arch.convs)
        conv_hi = (conv_hi + 3) // 4 * 4
        zero_in_head = B <= 32 and not self.two_stream
        # Two streams (= two parallel branches of the captured HIP graph):
        # main: forward -> head -> fc/conv3/conv2 dgrad chain (critical path)
        # side: grad zeroing (overlaps the forward) and every weight-gradient
        #       kernel, each gated on the dgrad output it consumes.
        # Measured on MI355X: the cross-stream waits cost more than the overlap
        # gains at B=32 (3.9k vs 4.5k steps/s), so the side branch is off by default.
        main = torch.cuda.current_stream(dev)
        side = self._side_stream(dev) if self.two_stream else main
        if not zero_in_head:
            side.wait_stream(main)
            with torch.cuda.stream(side):
                grad_out.zero_()
            ev_zero = self._event('zero', side)
        spec = batch.get('sample_spec')
        if spec is not None:
            assert self.fused_trunk and frames is not None, 'deferred sampling needs the fused trunk'
        sample = (spec, ninst) if spec is not None else None
        fold = self.can_fold_head(B, 0 if acting is None else E)
        # the fc / conv3 / conv2 dgrads as one launch (single-process grouped-wgrad path); its
        # counters are zeroed by this step's fc forward launch
        chain = (self.can_chain_dgrad(B) and not split and lowrank is None and B <= 32
                 and self.arch.network == 'nature')
        self._fc_zero = self._chain_ws(B, dev) if chain else None
        if acting is None:
            self._fwd_trunk(xs, packs, flats, ws, B, ninst, frames=frames, sample=sample, fc=not fold)
        else:
            self._fwd_trunk(xs + [acting['stacks']], packs + [po], flats + [eo], ws, B, ninst + 1, frames=frames,
                            M=[B] * ninst + [E], sample=sample, fc=not fold)
        if not zero_in_head:
            main.wait_event(ev_zero)
        det = bool(det_wgrad)
        assert not det or (self.can_det_wgrad(B) and lowrank is None), 'det_wgrad: not available here'
        zero = [grad_out.data_ptr() + 4 * conv_lo, conv_hi - conv_lo] if zero_in_head and not det else []
        # ---- fused head + TD loss + head backward
        w, b, wv, bv = self._head_ptrs(flats)
        g = lambda n: grad_out.data_ptr() + 4 * lay.offsets[n]
        if self.dueling:
            dw, db, dwv, dbv = g('advantage/output/w'), g('advantage/output/b'), g('value/output/w'), \
                g('value/output/b')
        else:
            dw, db, dwv, dbv = g('output/w'), g('output/b'), 0, 0
        act = batch['actions']
        assert act.dtype == torch.int32 and act.numel() == B
        rew, done, gam = (batch['rewards'].contiguous(), batch['dones'].contiguous(),
                          batch['gammas'].contiguous())
        wts = batch.get('weights')
        self._c51_dev = dev
        hints = [B, self.A, self.HID, int(self.dueling), int(self.huber), 0]
        hio = [act.data_ptr(), rew.data_ptr(), done.data_ptr(), gam.data_ptr(),
               wts.data_ptr() if wts is not None else 0, ws['loss'].data_ptr(), ws['prio'].data_ptr(),
               ws['q'].data_ptr() if not self.dist else 0, dw, db, dwv, dbv, ws['dh'].data_ptr()]
        hactor = [] if acting is None else list(acting['ptrs']) + list(acting['ints'])
        hactor_f = [] if acting is None else list(acting['f'])
        act_h = 0 if acting is None else ws['h'][ninst].data_ptr()
        if fold:
            # fc forward + output layer + TD loss + dQ / dH (+ the fused acting step): one launch
            self._fc_head(packs if acting is None else packs + [po], ws, B, ninst, hints, w, b, wv, bv, hio,
                          hactor, hactor_f, act_h, dev)
        else:
            self._head(hints, [ws['h'][i].data_ptr() for i in range(ninst)], w, b, wv, bv, hio,
                       *self._head_packs(packs), [],          # (the conv grad range is zeroed by the fc dgrad)
                       hactor, hactor_f, act_h=act_h, ws=ws)
        self._fc_zero = None                # (consumed by this step's fc forward launch)
        # ---- backward (online instance 0 only)
        c1, c2, c3 = self.arch.convs
        (h1, w1), (h2, w2), (h3, w3) = c1.out_hw, c2.out_hw, c3.out_hw
        H, HH, F = self.HID, self.HH, self.FLAT
        pko = lambda key: po.data_ptr() + self.esz * self.poff[key]
        if self.dueling:
            fw, fb, fw2, fb2 = g('value/fcl/w'), g('value/fcl/b'), g('advantage/fcl/w'), g('advantage/fcl/b')
        else:
            fw, fb, fw2, fb2 = g('fcl/w'), g('fcl/b'), 0, 0
        # fc dgrad (+ the scalar head's backward: dH, dW_out, db_out from the head's dQ)
        hmembers, hdims = self._head_wgrad_members(ws, B, ws['h'][0].data_ptr(), (dw, db, dwv, dbv))
        fc_dgrad = lambda: self._fc_dgrad(ws, B, po, zero, draw_noise)
        if self.arch.network == 'cnn':
            defer = bool(defer_fc) and self.can_defer_fc(B, gnoise is not None)
            assert defer or not defer_fc, 'defer_fc: not available for this executor / batch'
            dwg = bool(defer_wgrad)
            assert not dwg or (defer and not split and self.can_defer_wgrad(B, gnoise is not None)), \
                'defer_wgrad (cnn): needs defer_fc, one process'
            out = self._cnn_backward(ws, B, s, frames, po, g, fw, fb, fw2, fb2, grad_out, gnoise, dev, fc_dgrad,
                                     hmembers, hdims, defer=defer, defer_wgrad=dwg)
            return out + (None,) if split else out
        x1, x2, x3 = ws['x1'][0].data_ptr(), ws['x2'][0].data_ptr(), ws['x3'][0].data_ptr()
        mc_fc = (B + 31) // 32 * 32
        K1, K2, K3 = c1.k * c1.k * c1.cin, c2.k * c2.k * c2.cin, c3.k * c3.k * c3.cin
        d1 = [B * h1 * w1, c1.cout, K1, 0, 0, 84, 84, h1, w1, 0, 0]
        kind1 = _KIND['C1']
        if frames is not None:
            d1 += [frames.data_ptr(), 84 * 84]
            kind1 = _KIND['F1']
        # (fc wgrad members are plain stores only while one 32-row M-chunk covers the batch)
        if self.grouped_wgrad and not self.two_stream and B <= 32:
            # dgrad chain: dz3 = (dh W_fc^T)*(x3>0) -> dz2 -> dz1, then ONE grouped launch for
            # the four weight gradients (conv1 first: the longest member)
            members = [[kind1, s.data_ptr(), ws['dz1'].data_ptr(), c1.cout, g('conv1/w'), g('conv1/b'), 0, 0,
                        c1.cout, c1.cout],
                       [_KIND['C3'], x2, ws['dz3'].data_ptr(), c3.cout, g('conv3/w'), g('conv3/b'), 0, 0, c3.cout,
                        c3.cout],
                       [_KIND['C2'], x1, ws['dz2'].data_ptr(), c2.cout, g('conv2/w'), g('conv2/b'), 0, 0, c2.cout,
                        c2.cout],
                       [_KIND['DFWD'], x3, ws['dh'].data_ptr(), HH, fw, fb, fw2, fb2, H, HH]] + hmembers
            dims = [d1, [B * h3 * w3, c3.cout, K3, 0, 0, h2, w2, h3, w3, 0, 0],
                    [B * h2 * w2, c2.cout, K2, 0, 0, h1, w1, h2, w2, 0, 0], [B, HH, F, 0, 0, 0, 0, 0, 0, 0, 0]] + hdims
            scales = [self.input_scale] + [1.0] * (len(members) - 1)
            if det:
                pl = self._det_plan(B, dev)
                for m, c in zip(members[:3], (c1, c3, c2)):
                    m += self._det_member(pl, c.name)
                self._parts_pending = (pl['jobs'], pl['buf'].data_ptr())
            noisy = self.noisy and gnoise is not None
            defer = bool(defer_fc) and self.can_defer_fc(B, gnoise is not None)
            assert defer or not defer_fc, 'defer_fc: not available for this executor / batch'
            dwg = bool(defer_wgrad)
            assert not dwg or (defer and not det and self.can_defer_wgrad(B, gnoise is not None)
                               and (not split or (lowrank is not None and self.dp_exchange is not None))), \
                'defer_wgrad: needs defer_fc, no det_wgrad; under DP the low-rank exchange and dp_exchange'
            if defer and not (split and lowrank is not None):
                # the optimizer launch forms dW_fc = x3^T dH from this rank's rows
                self._fc_pending = (x3, ws['dh'].data_ptr(), B)
                members, dims, scales = members[:3] + members[4:], dims[:3] + dims[4:], scales[:3] + scales[4:]
            if split and not noisy and lowrank is not None:
                # (noisy nets reach here only with the sigma gradients left to the fused optimizer)
                assert self.lowrank_spec(B, sigma_fused=True) is not None, 'low-rank exchange not available here'
                W, rk = int(lowrank['world']), int(lowrank['rank'])
                lw = self._lowrank_ws(B, W, dev)
                if self.dist:                              # C51: dH = dlogits [W | Wv]^T * (h > 0) first
                    self._c51_dh(ws, B, po)
                # in stream order (a graph fork / join costs ~25 us on this ROCm: measured,
                # scripts/probe_graph_concurrency.py), right after the head: x3 and dh are final.
                # The all-gather runs as a side duty of the fc dgrad launch (its own grid.z slice)
                # when the transport can hand out device args; else as its own launch first.
                seg = ([x3, ws['dh'].data_ptr()], [lw['x'].data_ptr(), lw['dh'].data_ptr()],
                       [B * F * self.esz, B * HH * self.esz])
                ga = None
                if lowrank.get('gather_args') is not None:
                    dev_args, nblk = lowrank['gather_args'](*seg)      # (cached by the transport)
                    ga = (dev_args.data_ptr(), nblk)
                    self._fc_dgrad(ws, B, po, zero, draw_noise, dh_done=True, gather=ga)
                else:
                    lowrank['gather'](*seg)
                if defer:
                    # the optimizer launch forms dW_fc and the fc bias gradient from all W*B rows
                    self._fc_pending = (lw['x'].data_ptr(), lw['dh'].data_ptr(), W * B)
                else:
                    # sum over all W*B rows in one block per weight tile (64-row chunks in a fixed
                    # order, no atomics: bit-identical on every rank)
                    ext.qnet_wgrad(_KIND['DLR'], lw['x'].data_ptr(), [W * B, HH, F, 0, 0, 0, 0, 0, 0, 0, 0],
                                   lw['dh'].data_ptr(), HH, fw, fb, fw2, fb2, H, HH, 64, 64, 128, 1.0, False,
                                   mloop=(W * B + 63) // 64, db_zero=rk != 0)
                if ga is None:
                    self._fc_dgrad(ws, B, po, zero, draw_noise, dh_done=True)
                # the output layer's members join the conv members in the tail's grouped launch
                members, dims, scales = members[:3] + members[4:], dims[:3] + dims[4:], scales[:3] + scales[4:]
            elif split and not noisy:
                assert not defer, 'defer_fc under data parallelism needs the low-rank exchange'
                fc_dgrad()
                # dense weight gradients now (they need only dh, dQ and x3 / h): the dense range is final
                ext.qnet_wgrad_group(members[3:], dims[3:], scales[3:])
                members, dims, scales = members[:3], dims[:3], scales[:3]
            elif not chain:
                fc_dgrad()
            d3 = [B * h2 * w2, c3.cin, c3.k * c3.k * c3.cout, c3.cin // 16, c3.cin, h2, w2, h3, w3, 0, 0]
            d2 = [B * h1 * w1, c2.cin, c2.k * c2.k * c2.cout, c2.cin // 16, c2.cin, h1, w1, h2, w2, 0, 0]

            def tail():
                if chain:
                    # fc dgrad (+ its side duties) -> conv3 dgrad -> conv2 dgrad: ONE launch
                    if self.dist:                   # C51: dH = dlogits [W | Wv]^T * (h > 0) first
                        self._c51_dh(ws, B, po)
                    dh, pk, dz3, x3m, dims0, aux0, auxf0 = self._fc_dgrad_args(ws, B, po, zero, draw_noise)
                    three = self.chain_dgrad >= 2       # (2: the conv2 dgrad inside the chain too)
                    ext.qnet_dgrad_chain(dh, pk, dz3, x3m, dims0, aux0, auxf0, pko('conv3/dgrad'),
                                         ws['dz2'].data_ptr(), x2, d3, pko('conv2/dgrad'),
                                         ws['dz1'].data_ptr() if three else 0, x1, d2,
                                         self._chain_ws(B, dev).data_ptr(), B)
                    if not three:
                        ext.qnet_igemm(_KIND['D2'], [ws['dz2'].data_ptr()], [pko('conv2/dgrad')], [],
                                       [ws['dz1'].data_ptr()], [x1], [1.0], d2)
                else:
                    ext.qnet_igemm(_KIND['D3'], [ws['dz3'].data_ptr()], [pko('conv3/dgrad')], [],
                                   [ws['dz2'].data_ptr()], [x2], [1.0], d3)
                    ext.qnet_igemm(_KIND['D2'], [ws['dz2'].data_ptr()], [pko('conv2/dgrad')], [],
                                   [ws['dz1'].data_ptr()], [x1], [1.0], d2)
                if dwg:                 # the next update_and_pack runs the group beside the fc update
                    self._wg_pending = (members, dims, scales)
                else:
                    ext.qnet_wgrad_group(members, dims, scales)
                if noisy:
                    ext.qnet_noisy_grad(grad_out.data_ptr(), gnoise.data_ptr(), self._noisy_jobs_on(dev).data_ptr(),
                                        len(self.noisy_jobs), self._noisy_max)

            if split and not noisy:
                return ws['loss'], ws['prio'], tail
            tail()
            return (ws['loss'], ws['prio'], None) if split else (ws['loss'], ws['prio'])
        # fc dgrad: dz3 = (dh W^T) * (x3 > 0) (scalar heads: dh itself is built in this launch)
        fc_dgrad()
        side.wait_event(self._event('dz3', main))
        with torch.cuda.stream(side):
            # fc wgrad: dW[F][HH] = x3^T dh, db = sum dh
            ext.qnet_wgrad(_KIND['DFWD'], x3, [B, HH, F, 0, 0, 0, 0, 0, 0, 0, 0], ws['dh'].data_ptr(), HH,
                           fw, fb, fw2, fb2, H, HH, mc_fc, 64, 128, 1.0, False)
            for m, d in zip(hmembers, hdims):           # output layer (B > 32: atomics on the zeroed grad)
                ext.qnet_wgrad(m[0], m[1], d, m[2], m[3], m[4], m[5], m[6], m[7], m[8], m[9], 32, 64, 64, 1.0, True)
        with torch.cuda.stream(side):
            ext.qnet_wgrad(_KIND['C3'], x2, [B * h3 * w3, c3.cout, K3, 0, 0, h2, w2, h3, w3, 0, 0],
                           ws['dz3'].data_ptr(), c3.cout, g('conv3/w'), g('conv3/b'), 0, 0, c3.cout, c3.cout,
                           128, 192, 64, 1.0, True)
        ext.qnet_igemm(_KIND['D3'], [ws['dz3'].data_ptr()], [pko('conv3/dgrad')], [], [ws['dz2'].data_ptr()], [x2],
                       [1.0], [B * h2 * w2, c3.cin, c3.k * c3.k * c3.cout, c3.cin // 16, c3.cin, h2, w2, h3, w3,
                               0, 0])
        side.wait_event(self._event('dz2', main))
        with torch.cuda.stream(side):
            ext.qnet_wgrad(_KIND['C2'], x1, [B * h2 * w2, c2.cout, K2, 0, 0, h1, w1, h2, w2, 0, 0],
                           ws['dz2'].data_ptr(), c2.cout, g('conv2/w'), g('conv2/b'), 0, 0, c2.cout, c2.cout,
                           128, 128, 64, 1.0, True)
        ext.qnet_igemm(_KIND['D2'], [ws['dz2'].data_ptr()], [pko('conv2/dgrad')], [], [ws['dz1'].data_ptr()], [x1],
                       [1.0], [B * h1 * w1, c2.cin, c2.k * c2.k * c2.cout, c2.cin // 16, c2.cin, h1, w1, h2, w2,
                               0, 0])
        # conv1: wgrad only (input scale folded in); last kernel of the step, on main
        ext.qnet_wgrad(kind1, s.data_ptr(), d1, ws['dz1'].data_ptr(), c1.cout, g('conv1/w'), g('conv1/b'), 0, 0,
                       c1.cout, c1.cout, 128, 256, 32, self.input_scale, True)
        if self.noisy and gnoise is not None:      # dL/dsigma from dL/dW_eff (in the mu slots)
            ext.qnet_noisy_grad(grad_out.data_ptr(), gnoise.data_ptr(), self._noisy_jobs_on(dev).data_ptr(),
                                len(self.noisy_jobs), self._noisy_max)
        main.wait_stream(side)
        return (ws['loss'], ws['prio'], None) if split else (ws['loss'], ws['prio'])


class HipCnnExecutor(HipExecutor):
    """The reference `cnn` (/root/reference/src/network.py:317-424) on HIP: fused
    per-sample forward (conv/ReLU/max-pool x3 with the activations in LDS) and
    backward (pool argmax routing + conv dgrads) kernels from csrc/kernels/cnn.hip,
    plus the shared fc / head / grouped-wgrad / optimizer / pack kernels."""

    fused_sampling = False          # cnn.hip's forward reads sampler-made slot tables

    def _workspace(self, B: int, dev) -> dict:
        key = (B, dev.index if dev.index is not None else 0)
        ws = self._ws.get(key)
        if ws is not None:
            return ws
        bf = dict(dtype=self.act_dtype, device=dev)
        f32 = dict(dtype=torch.float32, device=dev)
        ws = {
            'x3': torch.zeros(4, B * self.FLAT, **bf),
            'h': torch.zeros(4, B * self.HH, **bf),
            'a1': torch.zeros(B * 441 * 32, **bf), 'p1': torch.zeros(B * 121 * 32, **bf),
            'a2': torch.zeros(B * 36 * 64, **bf), 'p2': torch.zeros(B * 9 * 64, **bf),
            'a3': torch.zeros(B * 9 * 64, **bf),
            'dh': torch.zeros(B * self.HH, **bf), 'dz3': torch.zeros(B * self.FLAT, **bf),
            'dc1': torch.zeros(B * 441 * 32, **bf), 'dc2': torch.zeros(B * 36 * 64, **bf),
            'dc3': torch.zeros(B * 9 * 64, **bf),
            'loss': torch.zeros(1, **f32), 'prio': torch.zeros(B, **f32), 'q': torch.zeros(B * self.A, **f32),
            'ones': torch.ones(B, **f32),
        }
        ws.update(self._head_ws(B, dev))
        self._ws[key] = ws
        return ws

    def _fwd_trunk(self, xs, packs, flats, ws, B, ninst, frames=None, keep_acts=True, M=(), sample=None, fc=True):
        assert sample is None, 'the cnn forward reads sampler-made slot tables'
        lay = self.layout
        pad = lambda v: list(v) + [0] * (4 - len(v))
        pk = lambda key: [p.data_ptr() + self.esz * self.poff[key] for p in packs]
        bias = lambda name: [f.data_ptr() + 4 * lay.offsets[name] for f in flats]
        slots = [x.data_ptr() for x in xs] if frames is not None else []
        states = [] if frames is not None else [x.data_ptr() for x in xs]
        keep = [ws[k].data_ptr() for k in ('a1', 'p1', 'a2', 'p2', 'a3')] if keep_acts else [0] * 5
        ptrs = (pad(slots) + pad(states) + pad(pk('conv1/fwd')) + pad(pk('conv2/fwd')) + pad(pk('conv3/fwd'))
                + pad(bias('conv1/b')) + pad(bias('conv2/b')) + pad(bias('conv3/b'))
                + pad([ws['x3'][i].data_ptr() for i in range(ninst)]) + keep)
        prof = self.cnn_prof[0].data_ptr() if self.cnn_prof is not None and keep_acts else 0
        self.ext.qnet_cnn_fwd(frames.data_ptr() if frames is not None else 0, ptrs, B, ninst, self.input_scale,
                              list(M), prof=prof)
        if fc:
            self._fc_fwd(packs, flats, ws, B, ninst)

    def _cnn_backward(self, ws, B, s, frames, po, g, fw, fb, fw2, fb2, grad_out, noise, dev, fc_dgrad,
                      hmembers=(), hdims=(), defer=False, defer_wgrad=False):
        ext = self.ext
        F, HH, H = self.FLAT, self.HH, self.HID
        pko = lambda key: po.data_ptr() + self.esz * self.poff[key]
        x3 = ws['x3'][0].data_ptr()
        # dp3 = (dh W_fc^T) * (pooled conv3 output > 0)
        fc_dgrad()
        # pool / ReLU / conv dgrad chain per sample -> d(conv pre-activations)
        ext.qnet_cnn_bwd([ws['dz3'].data_ptr(), ws['a1'].data_ptr(), ws['a2'].data_ptr(), ws['a3'].data_ptr(),
                          pko('conv3/dgrad'), pko('conv2/dgrad'), ws['dc1'].data_ptr(), ws['dc2'].data_ptr(),
                          ws['dc3'].data_ptr()], B,
                         prof=self.cnn_prof[1].data_ptr() if self.cnn_prof is not None else 0,
                         parts=self.tuning.cnn_parts(self.compute_dtype))
        c1, c2, c3 = self.arch.convs
        t1, _, l1, _ = c1.pads()
        t2, _, l2, _ = c2.pads()
        t3, _, l3, _ = c3.pads()
        d1 = [B * 441, c1.cout, c1.k * c1.k * c1.cin, 0, 0, 84, 84, 21, 21, t1, l1]
        kind1 = _KIND['C1']
        if frames is not None:
            d1 += [frames.data_ptr(), 84 * 84]
            kind1 = _KIND['F1']
        members = [[kind1, s.data_ptr(), ws['dc1'].data_ptr(), c1.cout, g('conv1/w'), g('conv1/b'), 0, 0, c1.cout,
                    c1.cout],
                   [_KIND['C3'], ws['p2'].data_ptr(), ws['dc3'].data_ptr(), c3.cout, g('conv3/w'), g('conv3/b'), 0, 0,
                    c3.cout, c3.cout],
                   [_KIND['C2'], ws['p1'].data_ptr(), ws['dc2'].data_ptr(), c2.cout, g('conv2/w'), g('conv2/b'), 0, 0,
                    c2.cout, c2.cout]]
        dims = [d1, [B * 9, c3.cout, c3.k * c3.k * c3.cin, 0, 0, 3, 3, 3, 3, t3, l3],
                [B * 36, c2.cout, c2.k * c2.k * c2.cin, 0, 0, 11, 11, 6, 6, t2, l2]]
        if defer:                       # dW_fc = x3^T dH inside the optimizer launch
            self._fc_pending = (x3, ws['dh'].data_ptr(), B)
        else:
            members.append([_KIND['DFWD'], x3, ws['dh'].data_ptr(), HH, fw, fb, fw2, fb2, H, HH])
            dims.append([B, HH, F, 0, 0, 0, 0, 0, 0, 0, 0])
        members += list(hmembers)
        dims += list(hdims)
        scales = [self.input_scale] + [1.0] * (len(members) - 1)
        if defer_wgrad:                 # the next update_and_pack runs the group beside the fc update
            self._wg_pending = (members, dims, scales)
        else:
            ext.qnet_wgrad_group(members, dims, scales)
        if self.noisy and noise is not None:
            ext.qnet_noisy_grad(grad_out.data_ptr(), noise.data_ptr(), self._noisy_jobs_on(dev).data_ptr(),
                                len(self.noisy_jobs), self._noisy_max)
        return ws['loss'], ws['prio']


def make_hip_executor(arch, layout, **kw):
    return (HipCnnExecutor if arch.network == 'cnn' else HipExecutor)(arch, layout, **kw)
