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

Transport: torch.distributed point-to-point (RCCL send/recv over xGMI on the GPU,
gloo on the CPU), one fp32 message each way per step: ``[n params (padded to even)]``
followed by a 2 x int64 header viewed in place (kind, value), so ``global_step`` travels
exactly (int64, not an fp32 that stops counting at 2^24).

  worker -> PS kinds: PUSH, PUSH_SYNC_TARGET (apply, then target <- online on the PS),
                      BYE (worker leaves)
  PS -> worker kinds: PARAMS, PARAMS_TARGET (a second message with the PS-owned target
                      follows), STOP (the PS is stopping: no more pushes)

``--disable_target_replication`` (reference `network.py:226-231`: the target variables
live on the PS): the PS owns the only target. A worker asks for the target sync at its own
cadence with PUSH_SYNC_TARGET (the reference's workers run the assign ops against the PS
target the same way, `dqn_agent.py:215-222`), and receives the PS target whenever it changed
since that worker last saw it. Without the flag each worker keeps its own replicated target.
"""
from __future__ import annotations

import contextlib
import logging
import time
from typing import Dict, Optional

import torch
import torch.distributed as dist

from .dist import DistContext

log = logging.getLogger(__name__)

PUSH, PUSH_SYNC_TARGET, BYE = 1, 2, -1
PARAMS, PARAMS_TARGET, STOP = 0, 3, 4


class _Msg:
    """fp32 payload + int64 (kind, value) header in one contiguous buffer."""

    def __init__(self, n: int, device):
        self.n = n
        self.pad = n + (n & 1)                  # 8-byte aligned header
        self.buf = torch.zeros(self.pad + 4, dtype=torch.float32, device=device)
        self.body = self.buf[:n]
        self.hdr = self.buf[self.pad:].view(torch.int64)

    def header(self):
        k, v = self.hdr.tolist()
        return int(k), int(v)


class AsyncPSServer:
    """Rank 0. ``net`` supplies the master parameters, gradient buffer, optimizer and (with
    ``own_target``) the PS-owned target."""

    def __init__(self, ctx: DistContext, network, own_target: Optional[bool] = None):
        assert ctx.enabled and ctx.rank == 0 and ctx.world_size >= 2, 'the PS is rank 0 of a world >= 2'
        self.ctx, self.net = ctx, network
        self.n = network.online.flat.numel()
        dev = network.online.flat.device
        if own_target is None:
            own_target = bool(getattr(network.config, 'disable_target_replication', False))
        self.own_target = own_target
        self.workers = list(range(1, ctx.world_size))
        self._in: Dict[int, _Msg] = {w: _Msg(self.n, dev) for w in self.workers}
        self._out: Dict[int, _Msg] = {w: _Msg(self.n, dev) for w in self.workers}
        self._tout: Dict[int, torch.Tensor] = ({w: torch.zeros(self.n, device=dev) for w in self.workers}
                                               if own_target else {})
        self._recv: Dict[int, object] = {}
        self._send: Dict[int, list] = {}
        # gloo completes a p2p receive only inside wait(), so there the server takes the
        # next push with ONE any-source receive; RCCL has no any-source receive, so there
        # it polls one posted irecv per worker (event queries)
        self._any_source = ctx.backend == 'gloo'
        self._any = _Msg(self.n, dev) if self._any_source else None
        self.updates = 0
        self.per_worker = {w: 0 for w in self.workers}
        self.target_version = 0
        self.target_syncs = 0
        self._seen_version = {w: -1 for w in self.workers}
        self.stopped_workers = 0

    def _reply(self, w: int, kind: int = PARAMS):
        for h in self._send.get(w) or []:
            h.wait()                          # the previous snapshot for w has left
        out = self._out[w]
        send_target = kind == PARAMS and self.own_target and self._seen_version[w] != self.target_version
        if send_target:
            kind = PARAMS_TARGET
        out.body.copy_(self.net.online.flat)
        out.hdr[0] = kind
        out.hdr[1:2].copy_(self.net.global_step.view(1))
        hs = [dist.isend(out.buf, dst=w)]
        if send_target:
            self._tout[w].copy_(self.net.target.flat)
            hs.append(dist.isend(self._tout[w], dst=w))
            self._seen_version[w] = self.target_version
        self._send[w] = hs

    def _post(self, w: int):
        if not self._any_source:
            self._recv[w] = dist.irecv(self._in[w].buf, src=w)

    def _next_push(self, active, idle_sleep: float):
        """(worker, message) of the next push to arrive."""
        if self._any_source:
            w = dist.recv(self._any.buf)
            return w, self._any
        while True:
            for w in sorted(active):
                req = self._recv[w]
                if req.is_completed():
                    req.wait()
                    return w, self._in[w]
            time.sleep(idle_sleep)

    def serve(self, max_updates: int = 0, idle_sleep: float = 1e-4, supervisor=None) -> int:
        """Apply pushes until every worker said goodbye (or max_updates). When ``supervisor``
        asks to stop, every worker's next push is answered with STOP instead of applied."""
        for w in self.workers:                # initial pull: every worker starts from the PS params
            self._reply(w)
            self._post(w)
        active = set(self.workers)
        while active and not (max_updates and self.updates >= max_updates):
            w, msg = self._next_push(active, idle_sleep)
            kind, _ = msg.header()
            if kind == BYE:
                active.discard(w)
                continue
            if supervisor is not None and supervisor.should_stop():
                self._reply(w, STOP)          # no further receive is posted for w
                active.discard(w)
                self.stopped_workers += 1
                continue
            # arrival-order apply: grad -> fused optimizer (global_step += 1 inside)
            self.net.grad.copy_(msg.body)
            self.net.apply_grads(1.0)
            if kind == PUSH_SYNC_TARGET and self.own_target:
                self.net.update_target(1.0)
                self.target_version += 1
                self.target_syncs += 1
            self.updates += 1
            self.per_worker[w] += 1
            self._reply(w)
            self._post(w)
            if supervisor is not None:
                supervisor.on_train_step(self.updates)
        for w in self.workers:
            for h in self._send.get(w) or []:
                h.wait()
        return self.updates


class AsyncPSClient:
    """Ranks >= 1: push the local gradient, pull the PS parameters (blocking pair)."""

    def __init__(self, ctx: DistContext, flat: torch.Tensor):
        assert ctx.enabled and ctx.rank >= 1
        self.ctx = ctx
        self.n = flat.numel()
        self._out = _Msg(self.n, flat.device)
        self._in = _Msg(self.n, flat.device)
        self.pushes = 0
        self.stopped = False           # the PS answered STOP: push nothing more
        self.target_updated = False    # the last pull also brought the PS-owned target

    def pull(self, flat: torch.Tensor, global_step: Optional[torch.Tensor] = None,
             target: Optional[torch.Tensor] = None):
        dist.recv(self._in.buf, src=0)
        kind, _ = self._in.header()
        if kind == STOP:
            self.stopped = True
            return
        flat.copy_(self._in.body)
        if global_step is not None:
            global_step.copy_(self._in.hdr[1:2].view_as(global_step))
        self.target_updated = False
        if kind == PARAMS_TARGET:
            if target is None:
                target = torch.empty_like(flat)       # keep the p2p sequence intact
            dist.recv(target, src=0)
            self.target_updated = True

    def exchange(self, grad: torch.Tensor, flat: torch.Tensor, global_step: Optional[torch.Tensor] = None,
                 sync_target: bool = False, target: Optional[torch.Tensor] = None) -> bool:
        """Push ``grad``, pull the parameters; False once the PS has said STOP."""
        if self.stopped:
            return False
        self._out.body.copy_(grad)
        self._out.hdr[0] = PUSH_SYNC_TARGET if sync_target else PUSH
        self._out.hdr[1] = self.pushes
        dist.send(self._out.buf, dst=0)
        self.pushes += 1
        self.pull(flat, global_step, target)
        return not self.stopped

    def close(self):
        if self.stopped:
            return                     # the PS already dropped this worker
        self._out.hdr[0] = BYE
        dist.send(self._out.buf, dst=0)


# ----------------------------------------------------------------------------------------------
# Transport over xGMI peer memory (csrc/kernels/async_ps.hip): one-sided device writes of the
# gradient into the PS's per-worker slot, device reads of the PS's per-worker parameter
# snapshot, control words in a host page shared by every rank and mapped into their GPUs.
_CTL_STRIDE = 128                     # bytes per worker: push word @0, done word @64
_BYE = 15                             # push kind: the worker leaves
_STOP_STATUS = 1                      # done status: the PS stopped


def ps_lowrank_plan(network, config) -> Optional[dict]:
    """--ps_lowrank (xgmi transport): the fc weight gradient travels as its factors -- the fc input
    rows X [B][F] and the dL/dh rows [B][HH] (act_t), rank <= B -- written into the slot where the
    fc weight gradient would be, instead of the 6.4 MB gradient (Nature, B = 32: ~0.56 MB pushed in all
    with the rest of the flat gradient). The server's fused optimizer launch forms dW = X^T dH from
    them (the single-process learner's FcFuse path), so the update is the same arithmetic. The same
    plan on every rank (decided from the config and the architecture). None when not applicable
    (noisy / distributional heads, B > 32, no fused fc path in this build)."""
    if not int(getattr(config, 'ps_lowrank', 1)):
        return None
    ex = network.executor
    B = int(config.minibatch_size)
    if (not hasattr(ex, 'can_defer_fc') or getattr(ex, 'noisy', False) or getattr(ex, 'dist', False)
            or not ex.can_defer_fc(B, True) or not hasattr(ex, 'update_and_pack')):
        return None
    lay = network.layout
    holes = sorted((lay.offsets[n], lay.offsets[n] + lay.numel(n)) for n in lay.names if n.endswith('fcl/w'))
    if not holes:
        return None
    esz = 2                                                   # act_t rows (16-bit builds: FcFuse)
    xbytes = B * int(ex.FLAT) * esz
    dbytes = B * int(ex.HH) * esz
    if xbytes % 16 or dbytes % 16 or 4 * (holes[0][1] - holes[0][0]) < xbytes + dbytes:
        return None
    keep, lo = [], 0                                          # the flat ranges outside the fc weights
    for a, b in holes:
        if a > lo:
            keep.append((lo, a))
        lo = b
    if lo < lay.total:
        keep.append((lo, lay.total))
    # (16-byte pieces: every kept range's start and length, and the factor slot's start, % 4 elements)
    if len(keep) + 2 > 6 or any((b - a) % 4 or a % 4 for a, b in keep) or holes[0][0] % 4:
        return None
    return {'B': B, 'keep': keep, 'x_off': 4 * holes[0][0], 'dh_off': 4 * holes[0][0] + xbytes,
            'xbytes': xbytes, 'dbytes': dbytes}


def _agree_lowrank(ctx: DistContext, plan: Optional[dict]):
    """The server and every worker must push / read the fc gradient the same way (factor rows or the
    fp32 gradient): gather every rank's plan over the control plane and fail on every rank together
    if they differ (a mismatch would read 16-bit factor rows as an fp32 gradient, or the reverse)."""
    key = None if plan is None else sorted((k, tuple(map(tuple, v)) if k == 'keep' else v) for k, v in plan.items())
    plans = ctx.ctrl_all_gather_object(key)
    if any(p != plans[0] for p in plans):
        raise ValueError('async PS: the low-rank push plan differs across ranks (%s); pass the network to '
                         'make_ps_client and use the same --ps_lowrank / --minibatch_size everywhere' % (plans,))


class _PSShared:
    """Rank 0's fine-grained HBM region ([W-1] gradient slots, [W-1] parameter snapshots, [W-1]
    int64 step words) exported over IPC, and the shared host control page, mapped by every rank."""

    def __init__(self, ctx: DistContext, n: int):
        import os
        import uuid

        import numpy as np
        from ..ops import _ext
        self.ext = ext = _ext.load(required=True)
        self.ctx, self.n = ctx, n
        self.W = ctx.world_size
        self.slot_bytes = (4 * n + 255) // 256 * 256
        nw = self.W - 1
        total = 2 * nw * self.slot_bytes + 64 * nw
        err, handle = None, None
        self.base, self.opened = 0, False
        if ctx.rank == 0:
            try:
                self.base = ext.xgmi_alloc(total)
                handle = ext.xgmi_ipc_handle(self.base)
            except Exception as e:  # noqa: BLE001
                err = e
        path = None
        if ctx.rank == 0 and err is None:
            shm = '/dev/shm' if os.path.isdir('/dev/shm') else '/tmp'
            path = os.path.join(shm, 'dqn_ps_ctl_%s' % uuid.uuid4().hex[:12])
        self.ctl_bytes = (self.W * _CTL_STRIDE + 4095) // 4096 * 4096
        if path is not None:
            try:
                np.memmap(path, dtype=np.uint8, mode='w+', shape=(self.ctl_bytes,))[:] = 0
            except Exception as e:  # noqa: BLE001
                err, path = e, None
        handle, path = ctx.ctrl_broadcast_object((handle, path))
        self.path = path
        self.ctl = None
        self.ctl_dev = 0
        if handle is not None and path is not None and err is None:
            try:
                self.ctl = np.memmap(path, dtype=np.uint8, mode='r+', shape=(self.ctl_bytes,))
                self.ctl_dev = ext.host_register(int(self.ctl.ctypes.data), self.ctl_bytes)
                if ctx.rank != 0:
                    self.base = ext.xgmi_ipc_open(handle)
                    self.opened = True
            except Exception as e:  # noqa: BLE001
                err = e
        ok = torch.tensor([0 if err is not None or handle is None else 1], dtype=torch.int32, device=ctx.device)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if int(ok) != 1:
            self.close()
            raise RuntimeError('async PS over xgmi: setup failed on some rank (here: %s)' % (err,))
        self.words = self.ctl.view(np.uint64)

    def slot(self, w: int) -> int:
        return self.base + (w - 1) * self.slot_bytes

    def snap(self, w: int) -> int:
        return self.base + (self.W - 1 + w - 1) * self.slot_bytes

    def snap_step(self, w: int) -> int:
        return self.base + 2 * (self.W - 1) * self.slot_bytes + 64 * (w - 1)

    def push_word(self, w: int, dev: bool = True):
        return (self.ctl_dev if dev else 0) + w * _CTL_STRIDE

    def done_word(self, w: int, dev: bool = True):
        return (self.ctl_dev if dev else 0) + w * _CTL_STRIDE + 64

    def read_push(self, w: int) -> int:
        return int(self.words[w * _CTL_STRIDE // 8])

    def read_done(self, w: int) -> int:
        return int(self.words[(w * _CTL_STRIDE + 64) // 8])

    def close(self):
        import os
        if self.ctl_dev:
            self.ext.host_unregister(int(self.ctl.ctypes.data))
            self.ctl_dev = 0
        self.ctl = None
        if self.opened:
            self.ext.xgmi_ipc_close(self.base)
            self.opened = False
        elif self.base:
            self.ext.xgmi_free(self.base)
        self.base = 0
        if self.ctx.rank == 0 and self.path:
            try:
                os.unlink(self.path)
            except FileNotFoundError:
                pass


class XgmiPSServer:
    """Rank 0 of ``--async_ps`` over xGMI peer memory: the same arrival-order semantics as
    `AsyncPSServer` (each push is applied with the fused optimizer to whatever the PS holds,
    then that worker gets the fresh parameters and int64 global_step), with no message copies:
    the optimizer reads the worker's gradient slot in place and one kernel writes the worker's
    snapshot and raises its done word. The host loop only polls the shared control page."""

    transport = 'xgmi'

    def __init__(self, ctx: DistContext, network, shared: Optional[_PSShared] = None):
        assert ctx.enabled and ctx.rank == 0 and ctx.world_size >= 2
        assert not getattr(network.config, 'disable_target_replication', False), \
            'the xgmi PS transport keeps replicated targets (use --ps_transport=p2p)'
        self.ctx, self.net = ctx, network
        self.lowrank = ps_lowrank_plan(network, network.config)
        self.n = network.online.flat.numel()
        self.sh = shared or _PSShared(ctx, self.n)
        _agree_lowrank(ctx, self.lowrank)
        self.workers = list(range(1, ctx.world_size))
        dev = network.online.flat.device
        self._grads = {w: self.sh.ext.tensor_from_ptr(self.sh.slot(w), self.n, dev.index or 0) for w in self.workers}
        self._ticket = torch.zeros(2, dtype=torch.int32, device=dev)
        self.updates = 0
        self.per_worker = {w: 0 for w in self.workers}
        self.stopped_workers = 0
        self.busy_s = 0.0

    def _apply(self, w: int):
        """Arrival-order update from worker w's slot, read in place (no repack: the server never runs
        the network). Low-rank pushes: the fused optimizer launch forms the fc gradient from the
        factors in the slot."""
        net = self.net
        if self.lowrank is None:
            net.apply_grads(1.0, grad=self._grads[w], repack=False)
            return
        base, lr = self.sh.slot(w), self.lowrank
        net.executor.update_and_pack(net.optimizer, net.online.flat, self._grads[w], 1.0, net.global_step,
                                     fc=(base + lr['x_off'], base + lr['dh_off'], lr['B']), pack=False)

    def _publish(self, w: int, seq: int, status: int = 0):
        st = status == 0
        self.sh.ext.ps_publish(self.sh.snap(w), self.net.online.flat if st else None, self.sh.snap_step(w),
                               self.net.global_step if st else None, self.sh.done_word(w), (seq << 4) | status,
                               self._ticket, self.n)

    def serve(self, max_updates: int = 0, idle_sleep: float = 2e-5, supervisor=None, native: bool = True) -> int:
        """Answer the workers' pushes until every worker left (or ``max_updates``). native: a C++
        thread (csrc/ps_server.cpp) polls the control page and replays one captured graph per
        push (fused optimizer on the slot in place + snapshot / step / done word); the Python
        thread only relays the supervisor (stop requests, step-count hooks). Otherwise the
        polling loop below, one eager optimizer + publish per push."""
        if native and hasattr(self.sh.ext, 'PsServer'):
            return self._serve_native(max_updates, supervisor)
        seen = {}
        for w in self.workers:                # initial pull (push number 1): the PS parameters
            self._publish(w, 1)
            seen[w] = 1
        active = set(self.workers)
        t_busy = time.perf_counter()
        while active and not (max_updates and self.updates >= max_updates):
            got = False
            for w in sorted(active):
                v = self.sh.read_push(w)
                s, kind = v >> 4, v & 15
                if s <= seen[w]:
                    continue
                got = True
                seen[w] = s
                if kind == _BYE:
                    active.discard(w)
                    continue
                if supervisor is not None and supervisor.should_stop():
                    self._publish(w, s, _STOP_STATUS)
                    active.discard(w)
                    self.stopped_workers += 1
                    continue
                # arrival-order apply, the gradient read in place from the worker's slot
                self._apply(w)
                self._publish(w, s)
                self.updates += 1
                self.per_worker[w] += 1
                if supervisor is not None:
                    supervisor.on_train_step(self.updates)
            if not got:
                time.sleep(idle_sleep)
        torch.cuda.synchronize(self.net.online.flat.device)
        self.busy_s = time.perf_counter() - t_busy
        self.net.refresh_packed()             # (updates ran without the repack)
        return self.updates

    def _serve_native(self, max_updates: int, supervisor) -> int:
        ext, sh, net = self.sh.ext, self.sh, self.net
        dev = net.online.flat.device
        for w in self.workers:                # initial pull (push number 1): the PS parameters
            self._publish(w, 1)
        if self.lowrank is not None:          # (no first-use allocations inside the capture)
            net.executor.prepare_update(net.optimizer, net.online.flat)
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        graphs = {}
        from ..utils.capture import quiet_capture
        with quiet_capture(), torch.cuda.stream(s):
            for w in self.workers:
                ga, gs = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
                with torch.cuda.graph(ga, stream=s, capture_error_mode='thread_local'):
                    # arrival-order apply, the gradient read in place from worker w's slot (no
                    # repack: the server never runs the network); the answer's push number comes
                    # from w's push word (the kernel echoes it)
                    self._apply(w)
                    ext.ps_publish(sh.snap(w), net.online.flat, sh.snap_step(w), net.global_step, sh.done_word(w), 0,
                                   self._ticket, self.n, echo=sh.push_word(w))
                with torch.cuda.graph(gs, stream=s, capture_error_mode='thread_local'):
                    ext.ps_publish(sh.snap(w), None, sh.snap_step(w), None, sh.done_word(w), _STOP_STATUS,
                                   self._ticket, self.n, echo=sh.push_word(w))
                graphs[w] = (ga, gs)
        self._native_graphs = graphs          # (alive while the server replays them)
        srv = ext.PsServer(int(sh.ctl.ctypes.data), len(self.workers), _CTL_STRIDE, s.cuda_stream, dev.index or 0)
        for w, (ga, gs) in graphs.items():
            srv.set_graphs(w, ga.raw_cuda_graph_exec(), gs.raw_cuda_graph_exec())
        srv.start(int(max_updates), 1)
        last = 0
        ck = getattr(supervisor, 'ckpt', None)

        @contextlib.contextmanager
        def paused():
            srv.pause()                       # the server thread drains its stream and waits
            try:
                yield
            finally:
                srv.resume()
        if ck is not None:
            ck.quiesce = paused               # periodic saves read one update's consistent state
        try:
            while srv.running():
                if supervisor is not None:
                    u = srv.updates()
                    if u != last:
                        last = u
                        supervisor.on_train_step(u)
                    if supervisor.should_stop():
                        srv.request_stop()
                time.sleep(1e-3)
        finally:
            if ck is not None:
                ck.quiesce = None
            self.updates = srv.wait()
        self.pauses = int(srv.pauses())
        self.marks = list(srv.marks()) if hasattr(srv, 'marks') else []   # (s at every 64th update)
        _, per, stopped, busy = srv.stats()
        self.per_worker = {w: int(per[w]) for w in self.workers}
        self.stopped_workers = int(stopped)
        self.busy_s = float(busy)
        torch.cuda.current_stream(dev).wait_stream(s)
        self.net.refresh_packed()             # (updates ran without the repack)
        torch.cuda.synchronize(dev)
        return self.updates

    def close(self):
        self.sh.close()


class XgmiPSClient:
    """Ranks >= 1 of ``--async_ps`` over xGMI: ``exchange`` enqueues the push (peer stores into
    the PS slot + push word) and the pull (wait for the done word, snapshot -> local parameters
    and global_step) on the current stream with no host synchronisation."""

    transport = 'xgmi'

    def __init__(self, ctx: DistContext, flat: torch.Tensor, shared: Optional[_PSShared] = None,
                 timeout_s: float = 60.0, pipeline: bool = False, lowrank: Optional[dict] = None):
        assert ctx.enabled and ctx.rank >= 1
        self.ctx, self.w = ctx, ctx.rank
        self.n = flat.numel()
        self.sh = shared or _PSShared(ctx, self.n)
        dev = flat.device
        self._seq = torch.ones(1, dtype=torch.int64, device=dev)      # push number 1 = the initial pull
        self._gate = torch.zeros(2, dtype=torch.int64, device=dev)
        self._err = torch.zeros(1, dtype=torch.int32, device=dev)
        self._stopped = torch.zeros(1, dtype=torch.int32, device=dev)
        self._ticket = torch.zeros(2, dtype=torch.int32, device=dev)
        self._empty = torch.zeros(0, dtype=torch.float32, device=dev)
        self.timeout_ns = int(timeout_s * 1e9)
        self.pushes = 0
        self.target_updated = False
        self._host_pushes = 1
        # pipelined exchange (--ps_pipeline): take the answer to the previous push, then push; the
        # server answered it while this worker computed the gradient, so the wait is usually over
        self.pipeline = bool(pipeline)
        self._flushed_at = -1                 # push count whose answer flush() took
        self.lowrank = lowrank                # ps_lowrank_plan: push the fc factors, not the fc gradient
        _agree_lowrank(ctx, lowrank)          # (the server's plan, checked on every rank)

    @property
    def stopped(self) -> bool:
        """The PS answered STOP (host read of the shared done word, no GPU sync)."""
        return (self.sh.read_done(self.w) & 15) == _STOP_STATUS

    def _pull(self, flat, global_step):
        step = global_step if global_step is not None else torch.zeros(1, dtype=torch.int64, device=flat.device)
        self.sh.ext.ps_pull(flat, self.sh.snap(self.w), step, self.sh.snap_step(self.w), self.sh.done_word(self.w),
                            self._seq, self._gate, self._err, self._stopped, self.timeout_ns)

    def pull(self, flat: torch.Tensor, global_step: Optional[torch.Tensor] = None, target=None):
        self._pull(flat, global_step)

    def exchange(self, grad: torch.Tensor, flat: torch.Tensor, global_step: Optional[torch.Tensor] = None,
                 sync_target: bool = False, target: Optional[torch.Tensor] = None, fc_rows=None) -> bool:
        if self.stopped:
            return False
        self.exchange_kernels(grad, flat, global_step, fc_rows)
        self.pushes += 1
        return True

    # the push / pull launches keep their sequence numbers on the device: a captured graph replays them
    in_graph = True

    def exchange_kernels(self, grad: torch.Tensor, flat: torch.Tensor, global_step: Optional[torch.Tensor] = None,
                         fc_rows=None):
        '''The exchange's launches only (graph-capturable; after a STOP answer the pull copies nothing
        and the push lands in a slot the server no longer reads). fc_rows (low-rank push): device
        pointers (X rows, dL/dh rows) of the deferred fc gradient.'''
        if self.pipeline:
            # answer to push k-1 -> parameters (this step's gradient is computed already: stream
            # order), then push k into the slot the server has finished reading (it answered k-1)
            self._pull(flat, global_step)
            self._push(grad, fc_rows)
        else:
            self._push(grad, fc_rows)
            self._pull(flat, global_step)

    def _push(self, grad, fc_rows):
        slot = self.sh.slot(self.w)
        if self.lowrank is None:
            self.sh.ext.ps_push(grad, slot, self.sh.push_word(self.w), self._seq, PUSH, self._ticket)
            return
        assert fc_rows is not None, 'low-rank push: the learner defers the fc gradient'
        lr, g = self.lowrank, grad.data_ptr()
        src = [g + 4 * a for a, _ in lr['keep']] + [int(fc_rows[0]), int(fc_rows[1])]
        dst = [slot + 4 * a for a, _ in lr['keep']] + [slot + lr['x_off'], slot + lr['dh_off']]
        nb = [4 * (b - a) for a, b in lr['keep']] + [lr['xbytes'], lr['dbytes']]
        self.sh.ext.ps_push_segs(src, dst, nb, self.sh.push_word(self.w), self._seq, PUSH, self._ticket)

    def flush(self, flat: torch.Tensor, global_step: Optional[torch.Tensor] = None) -> bool:
        '''Pipelined exchange: take the answer to the last push (the parameters after it) into
        ``flat`` -- a worker's parameters otherwise lag one PS answer behind at the end of training
        (Learner.finish_ps). Returns whether it pulled.'''
        if self.pipeline and not self.stopped and self.pushes > 0 and self._flushed_at != self.pushes:
            self._pull(flat, global_step)
            self._flushed_at = self.pushes
            return True
        return False

    def check(self) -> bool:
        """False if a pull timed out waiting for the PS (host sync)."""
        return int(self._err[0]) == 0

    def close(self):
        if self.pipeline and not self.stopped and self.pushes > 0 and self._flushed_at != self.pushes:
            # the server must answer the last gradient push before BYE replaces it in the push word
            # (unless flush() already took that answer)
            scratch = torch.empty(self.n, dtype=torch.float32, device=self._seq.device)
            self._pull(scratch, None)
        if not self.stopped:
            self.sh.ext.ps_push(self._empty, self.sh.slot(self.w), self.sh.push_word(self.w), self._seq, _BYE,
                                self._ticket)
        torch.cuda.synchronize(self._seq.device)
        self.sh.close()


def ps_transport(ctx: DistContext, config) -> str:
    """'xgmi' or 'p2p' for --async_ps (identical on every rank: decided from the config)."""
    want = getattr(config, 'ps_transport', 'auto')
    if want == 'p2p' or ctx.device.type != 'cuda' or getattr(config, 'disable_target_replication', False):
        return 'p2p'
    return 'xgmi'


def make_ps_server(ctx: DistContext, network, config):
    if ps_transport(ctx, config) == 'xgmi':
        try:
            return XgmiPSServer(ctx, network)
        except RuntimeError as e:
            log.warning('async PS over xgmi unavailable (%s): torch.distributed p2p instead', e)
    return AsyncPSServer(ctx, network)


def make_ps_client(ctx: DistContext, flat: torch.Tensor, config, network=None):
    """``network``: the worker's Network -- its low-rank push plan is decided here and checked
    against the server's (required for the xgmi transport's --ps_lowrank)."""
    if ps_transport(ctx, config) == 'xgmi':
        try:
            return XgmiPSClient(ctx, flat, timeout_s=float(getattr(config, 'ps_timeout_s', 60.0)),
                                pipeline=bool(getattr(config, 'ps_pipeline', 0)),
                                lowrank=ps_lowrank_plan(network, config) if network is not None else None)
        except RuntimeError as e:
            log.warning('async PS over xgmi unavailable (%s): torch.distributed p2p instead', e)
    return AsyncPSClient(ctx, flat)
