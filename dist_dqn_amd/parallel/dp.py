"""Synchronous data parallelism (replaces the reference's parameter server,
`/root/reference/src/network.py:184-202` and `/root/reference/src/main.py:105-121`).

Every rank holds the online AND target parameters in HBM. Per SGD step the
flat gradient buffer is summed across ranks and every rank applies the same
fused optimizer update with ``grad_scale = 1/world`` folded into the kernel,
so parameters stay bit-identical without any parameter traffic (reference
messages M1/M2/M4/M6 disappear; only M3 = one gradient all-reduce remains).

Transports (``--allreduce``):
  * ``rccl``  — ``torch.distributed`` all_reduce (RCCL over xGMI; gloo on the CPU),
    issued between HIP-graph segments.
  * ``xgmi``  — the peer-to-peer kernel of `parallel/xgmi.py` (IPC-mapped peer
    buffers, two-shot over the point-to-point links); a plain launch, so the whole
    step including both all-reduces stays ONE captured HIP graph.
  * ``auto``  (default) — on GPUs, set up ``xgmi``, self-test it, time both on the
    real gradient size and keep the faster (decided on rank 0, same on every rank);
    RCCL whenever xgmi cannot be set up or fails its self-test.

Gradient message sizing for xGMI: the reference `cnn` is
0.58 MB fp32, Nature-CNN 6.7 MB (95% of it the FC layer). ``--allreduce_dtype=bf16``
sends bf16 on the wire (fp32 master gradient kept; every rank ends with the same
bf16-rounded sum).
"""
from __future__ import annotations

import logging
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

from .dist import DistContext

log = logging.getLogger(__name__)


class GradAllReducer:
    def __init__(self, ctx: DistContext, flat_grad: torch.Tensor, bucket_mb: float = 64.0,
                 mode: str = 'auto', wire_dtype: str = 'fp32', gather_bytes: int = 0, exchange_slots: int = 0):
        self.ctx = ctx
        self.flat = flat_grad
        n = flat_grad.numel()
        per = max(1, int(bucket_mb * 1024 * 1024 / flat_grad.element_size()))
        per = (per + 63) // 64 * 64
        self.buckets: List[Tuple[int, int]] = [(o, min(n, o + per)) for o in range(0, n, per)]
        self.comm_stream = (torch.cuda.Stream(device=flat_grad.device)
                            if flat_grad.is_cuda and ctx.enabled else None)
        assert mode in ('rccl', 'xgmi', 'auto'), mode
        self.requested = mode
        self.wire_dtype = wire_dtype
        self.wire = None
        if wire_dtype == 'bf16' and ctx.enabled:
            self.wire = torch.zeros(n, dtype=torch.bfloat16, device=flat_grad.device)
        self.xgmi = None
        self.timings = {}
        self.gather_bytes = int(gather_bytes)
        # > 0: the xgmi transport also carries the fused update's in-launch exchange channel
        # (learner.py: the conv / output-layer gradients summed inside the update launch)
        self.exchange_slots = int(exchange_slots)
        self.can_gather = False       # the xgmi transport carries a working all-gather channel
        self.can_exchange = False     # ... and a working in-launch update-exchange channel
        if ctx.enabled and flat_grad.is_cuda and mode in ('xgmi', 'auto'):
            self.xgmi = self._setup_xgmi(mode)
        self.mode = 'xgmi' if self.xgmi is not None else 'rccl'

    # ------------------------------------------------------------ transport choice
    def _setup_xgmi(self, mode: str):
        from .xgmi import XgmiAllReduce
        n = self.flat.numel()
        try:
            x = XgmiAllReduce(self.ctx, n, self.wire_dtype, gather_bytes=self.gather_bytes,
                              exchange_slots=self.exchange_slots)
        except Exception as e:  # noqa: BLE001
            if mode == 'xgmi':
                raise
            log.warning('xgmi all-reduce unavailable (%s); using RCCL', e)
            return None
        if not x.self_test(n):
            x.close()
            if mode == 'xgmi':
                raise RuntimeError('xgmi all-reduce failed its self-test')
            log.warning('xgmi all-reduce failed its self-test; using RCCL')
            return None
        if self.gather_bytes > 0:
            self.can_gather = x.self_test_gather()
            if not self.can_gather:
                log.warning('xgmi all-gather failed its self-test; dense gradients all-reduced in full')
        # the fused update's in-launch exchange channel: its own protocol self-test (a failure keeps
        # the transport, without the fused DP step: the learner then all-reduces between launches)
        self.can_exchange = bool(self.exchange_slots > 0 and x.self_test_dpx())
        if self.exchange_slots > 0 and not self.can_exchange:
            log.warning('xgmi update-exchange failed its self-test; the DP step keeps a separate all-reduce')
        agree = self._cross_check(x)
        if not agree:
            x.close()
            if mode == 'xgmi':
                raise RuntimeError('xgmi all-reduce disagrees with RCCL on the gradient buffer')
            log.warning('xgmi all-reduce disagrees with RCCL on the gradient buffer; using RCCL')
            return None
        if mode == 'auto':
            t_x = self._time(lambda t: x.allreduce(t, 0))
            t_r = self._time(lambda t: dist.all_reduce(t, op=dist.ReduceOp.SUM))
            self.timings.update(xgmi_us=t_x, rccl_us=t_r)
            if self.ctx.is_chief:
                log.info('gradient all-reduce (%d elems): xgmi %.1f us, rccl %.1f us', n, t_x, t_r)
            # (with a working gather channel the learner all-reduces only the small non-factored
            # range over xgmi and exchanges the dense factors: far fewer bytes than either
            # full-buffer time measured here, so xgmi is kept)
            if t_x > t_r and not self.can_gather:
                x.close()
                return None
        return x

    def _cross_check(self, x) -> bool:
        """Start-up consistency check on the real gradient size: the xgmi sum of random
        gradients must match RCCL's (to summation-order rounding: fp32 1e-5 relative, bf16 wire
        2e-2) and be bit-identical on every rank (the replicas' invariant). Agreed on all ranks."""
        n = self.flat.numel()
        g = torch.Generator(device=self.flat.device).manual_seed(1234 + self.ctx.rank)
        t = torch.randn(n, generator=g, device=self.flat.device)
        a, b = t.clone(), t.clone()
        x.allreduce(a, 0)
        dist.all_reduce(b, op=dist.ReduceOp.SUM)
        ref = a.clone()
        dist.broadcast(ref, src=0)
        rel = float(((a - b).abs().max() / b.abs().max().clamp_min(1e-30)))
        tol = 2e-2 if self.wire_dtype == 'bf16' else 1e-5
        ok = torch.tensor([1 if (rel <= tol and torch.equal(ref, a) and x.check()) else 0], dtype=torch.int32,
                          device=self.flat.device)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        self.timings['xgmi_vs_rccl_max_rel'] = rel
        return bool(int(ok))

    def _time(self, fn, iters: int = 20) -> float:
        """Mean us per call over ``iters`` (after 3 warm-up calls), max over ranks."""
        t = torch.zeros_like(self.flat)
        for _ in range(3):
            fn(t)
        self.ctx.barrier()
        torch.cuda.synchronize(self.flat.device)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn(t)
        e1.record()
        torch.cuda.synchronize(self.flat.device)
        us = torch.tensor([1000.0 * e0.elapsed_time(e1) / iters], dtype=torch.float64, device=self.flat.device)
        dist.all_reduce(us, op=dist.ReduceOp.MAX)
        return float(us)

    @property
    def in_graph(self) -> bool:
        """True when the all-reduce is a plain kernel launch (capturable in the step graph)."""
        return self.xgmi is not None

    @property
    def scale(self) -> float:
        return 1.0 / self.ctx.world_size

    # --------------------------------------------------------------- collectives
    def allreduce(self):
        """Blocking (stream-ordered) sum of the whole flat gradient."""
        if not self.ctx.enabled:
            return
        if self.xgmi is not None:
            self.xgmi.allreduce(self.flat, 0)
            return
        if self.wire is not None:
            self.wire.copy_(self.flat)
            for lo, hi in self.buckets:
                dist.all_reduce(self.wire[lo:hi], op=dist.ReduceOp.SUM)
            self.flat.copy_(self.wire)
            return
        for lo, hi in self.buckets:
            dist.all_reduce(self.flat[lo:hi], op=dist.ReduceOp.SUM)

    def allreduce_range(self, lo: int, hi: int, channel: int = 0):
        """xgmi: sum of flat[lo:hi] on the current stream (graph-capturable); channels 0/1
        may run concurrently on different streams."""
        assert self.xgmi is not None
        if hi > lo:
            self.xgmi.allreduce(self.flat[lo:hi], channel)

    def allreduce_range_async(self, lo: int, hi: int):
        """Start the sum of flat[lo:hi] (whole range, one collective); returns a handle for
        ``wait_all``. RCCL runs it on its own stream, ordered after the work already queued on the
        current stream, so the kernels queued next overlap it."""
        if not self.ctx.enabled or hi <= lo:
            return None
        if self.wire is not None:
            w = self.wire[lo:hi]
            w.copy_(self.flat[lo:hi])
            return (dist.all_reduce(w, op=dist.ReduceOp.SUM, async_op=True), lo, hi)
        return (dist.all_reduce(self.flat[lo:hi], op=dist.ReduceOp.SUM, async_op=True), lo, hi)

    def wait_all(self, handles):
        """Make the current stream wait for the started range all-reduces (no host sync)."""
        for h in handles:
            if h is None:
                continue
            work, lo, hi = h
            work.wait()
            if self.wire is not None:
                self.flat[lo:hi].copy_(self.wire[lo:hi])

    def check(self):
        """Raise if the xgmi transport reported a timed-out peer wait (host sync)."""
        if self.xgmi is not None and not self.xgmi.check():
            raise RuntimeError('xgmi all-reduce: a peer wait timed out (rank %d: %s)'
                               % (self.ctx.rank, self.xgmi.error_info()))

    def close(self):
        if self.xgmi is not None:
            self.xgmi.close()
            self.xgmi = None


def broadcast_flat(ctx: DistContext, flat: torch.Tensor, src: int = 0):
    """One flat buffer from ``src`` to every rank."""
    if ctx.enabled:
        dist.broadcast(flat, src=src)


def state_tensors(net) -> List[Tuple[str, torch.Tensor]]:
    """Every device tensor that must be identical on all sync-DP replicas: online and target
    parameters, every optimizer slot, Adam's beta powers, the device global_step and, for
    noisy nets, the current noise samples and the device Philox state that draws the next."""
    out = [('online', net.online.flat), ('target', net.target.flat), ('global_step', net.global_step)]
    out += [('slot/%s' % n, s) for n, s in zip(net.optimizer.slot_names(), net.optimizer.slots)]
    out.append(('beta_powers', net.optimizer.beta_powers))
    for name in ('noise', 'noise_target', 'noise_rng'):
        t = getattr(net, name, None)
        if t is not None:
            out.append((name, t))
    return out


def broadcast_state(ctx: DistContext, net, src: int = 0):
    """Reference M8 (Supervisor init / restore, `/root/reference/src/main.py:136-143,155`): the
    chief's initialised or restored state reaches every rank — parameters, target, optimizer
    slots, beta powers, global_step and the noise stream — and every rank then rebuilds its
    packed MFMA fragments (noisy nets: re-mixed under the broadcast noise)."""
    if not ctx.enabled:
        return
    for _, t in state_tensors(net):
        dist.broadcast(t, src=src)
    net.refresh_packed()


def check_state_equal(ctx: DistContext, net) -> dict:
    """{tensor name: bit-equal to rank 0 on every rank} over `state_tensors` (host sync)."""
    out = {}
    for name, t in state_tensors(net):
        if not ctx.enabled:
            out[name] = True
            continue
        ref = t.clone()
        dist.broadcast(ref, src=0)
        same = torch.tensor([1 if torch.equal(ref, t) else 0], dtype=torch.int32, device=t.device)
        dist.all_reduce(same, op=dist.ReduceOp.MIN)
        out[name] = bool(int(same))
    return out


def check_replicas_equal(ctx: DistContext, flat: torch.Tensor) -> bool:
    """Debug/test helper: max |param - rank0 param| == 0 on every rank."""
    if not ctx.enabled:
        return True
    ref = flat.clone()
    dist.broadcast(ref, src=0)
    diff = (ref - flat).abs().max().view(1)
    dist.all_reduce(diff, op=dist.ReduceOp.MAX)
    return float(diff) == 0.0
