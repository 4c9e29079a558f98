"""Asynchronous parameter-server emulation (the reference's default mode).

Reference: without ``--sync`` every worker computes gradients on its own
minibatch and applies them to the PS-held variables with no locking
(between-graph replication, Hogwild-style; `/root/reference/src/main.py:105-129`,
`/root/reference/src/network.py:184-202`). The global
step is shared; workers read whatever parameters the PS holds at that moment.

Here (``--async_ps``) rank 0 is the parameter server, like the reference's
dedicated PS process (``dqn_multi_gpu.sh`` leaves GPU 0 to it): it owns the
master parameters and the optimizer state in its HBM and applies each worker's
gradient push IN ARRIVAL ORDER with the fused optimizer kernel, then answers
that worker with the fresh parameters and global step. Workers (ranks >= 1)
never wait for each other, so a push is applied to parameters other workers
have moved since that worker's pull: the same staleness as the reference.
Transport is torch.distributed point-to-point (RCCL send/recv over xGMI on
the GPU, gloo on the CPU): one ``[n + 1]`` fp32 message each way per step,
the extra slot carrying a header (push: +1 / goodbye: -1; reply: global step).
"""
from __future__ import annotations

import logging
import time
from typing import Dict, Optional

import torch
import torch.distributed as dist

from .dist import DistContext

log = logging.getLogger(__name__)

PUSH, BYE = 1.0, -1.0


class AsyncPSServer:
    """Rank 0. ``net`` supplies the master parameters, gradient buffer and optimizer."""

    def __init__(self, ctx: DistContext, network):
        assert ctx.enabled and ctx.rank == 0 and ctx.world_size >= 2, 'the PS is rank 0 of a world >= 2'
        self.ctx, self.net = ctx, network
        self.n = network.online.flat.numel()
        dev = network.online.flat.device
        self.workers = list(range(1, ctx.world_size))
        self._in: Dict[int, torch.Tensor] = {w: torch.zeros(self.n + 1, device=dev) for w in self.workers}
        self._out: Dict[int, torch.Tensor] = {w: torch.zeros(self.n + 1, device=dev) for w in self.workers}
        self._recv: Dict[int, object] = {}
        self._send: Dict[int, object] = {}
        # gloo completes a p2p receive only inside wait(), so there the server takes the
        # next push with ONE any-source receive; RCCL has no any-source receive, so there
        # it polls one posted irecv per worker (event queries)
        self._any_source = ctx.backend == 'gloo'
        self._any = torch.zeros(self.n + 1, device=dev) if self._any_source else None
        self.updates = 0
        self.per_worker = {w: 0 for w in self.workers}

    def _reply(self, w: int):
        if self._send.get(w) is not None:
            self._send[w].wait()              # the previous snapshot for w has left
        out = self._out[w]
        out[:self.n].copy_(self.net.online.flat)
        out[self.n:].copy_(self.net.global_step.to(out.dtype).view(1))
        self._send[w] = dist.isend(out, dst=w)

    def _next_push(self, active, idle_sleep: float):
        """(worker, message) of the next push to arrive."""
        if self._any_source:
            w = dist.recv(self._any)
            return w, self._any
        while True:
            for w in sorted(active):
                req = self._recv[w]
                if req.is_completed():
                    req.wait()
                    return w, self._in[w]
            time.sleep(idle_sleep)

    def serve(self, max_updates: int = 0, idle_sleep: float = 1e-4) -> int:
        """Apply pushes until every worker said goodbye (or max_updates)."""
        for w in self.workers:                # initial pull: every worker starts from the PS params
            self._reply(w)
            if not self._any_source:
                self._recv[w] = dist.irecv(self._in[w], src=w)
        active = set(self.workers)
        while active and not (max_updates and self.updates >= max_updates):
            w, msg = self._next_push(active, idle_sleep)
            if float(msg[self.n]) == BYE:
                active.discard(w)
                continue
            # arrival-order apply: grad -> fused optimizer (global_step += 1 inside)
            self.net.grad.copy_(msg[:self.n])
            self.net.apply_grads(1.0)
            self.updates += 1
            self.per_worker[w] += 1
            self._reply(w)
            if not self._any_source:
                self._recv[w] = dist.irecv(self._in[w], src=w)
        for w in self.workers:
            if self._send.get(w) is not None:
                self._send[w].wait()
        return self.updates


class AsyncPSClient:
    """Ranks >= 1: push the local gradient, pull the PS parameters (blocking pair)."""

    def __init__(self, ctx: DistContext, flat: torch.Tensor):
        assert ctx.enabled and ctx.rank >= 1
        self.ctx = ctx
        self.n = flat.numel()
        self._out = torch.zeros(self.n + 1, device=flat.device)
        self._in = torch.zeros(self.n + 1, device=flat.device)
        self.pushes = 0

    def pull(self, flat: torch.Tensor, global_step: Optional[torch.Tensor] = None):
        dist.recv(self._in, src=0)
        flat.copy_(self._in[:self.n])
        if global_step is not None:
            global_step.copy_(self._in[self.n:].to(global_step.dtype).view_as(global_step))

    def exchange(self, grad: torch.Tensor, flat: torch.Tensor, global_step: Optional[torch.Tensor] = None):
        self._out[:self.n].copy_(grad)
        self._out[self.n] = PUSH
        dist.send(self._out, dst=0)
        self.pushes += 1
        self.pull(flat, global_step)

    def close(self):
        self._out[self.n] = BYE
        dist.send(self._out, dst=0)
