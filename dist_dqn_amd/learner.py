"""Device-resident learner step (reference `DQNAgent._train_minibatch`,
`/root/reference/src/dqn_agent.py:108-143`).

Reference per step: python `random.sample` over a deque, host partition,
`session.run(target_q_output)` (H2D of next states, D2H of Q), host max,
python loop building y / one-hot, `session.run(train_op)` (H2D 3.6 MB feed),
optional summary, optional target assign — two host round trips per step.

Here one step is, entirely on the GPU and with no host synchronisation:
  sample (uniform w/o replacement, or PER sum-tree)  ->  gather uint8 stacks
  -> online fwd(s) + target fwd(s') [+ online fwd(s') for Double DQN]
  -> fused TD loss (+dQ)  ->  backward into the flat grad buffer
  -> [RCCL all-reduce of the flat grad]  ->  fused optimizer (+global_step++)
  -> [PER priority update]  ->  target copy/Polyak behind a device predicate.
On the GPU the sequence is captured once into a HIP graph (via
``torch.cuda.CUDAGraph``, which is hipGraph on ROCm) and replayed, so the
per-step host cost is one graph launch. With world > 1 the collective sits
between two captured graphs (pre: sample..backward, post: optimizer..target).
"""
from __future__ import annotations

import logging
from typing import Dict, Optional

import torch

from .models.network import Network
from .ops import kernels
from .parallel.dist import DistContext
from .parallel.dp import GradAllReducer
from .utils.capture import quiet_capture
from .utils.trace import trace

log = logging.getLogger(__name__)



_CAPTURE_MODE = 'thread_local'

def _reduce_ranges(layout, total: int, excluded, forbidden=(), max_ranges: int = 8):
    """The pieces of the flat gradient a data-parallel step still all-reduces: every layout
    tensor not inside an ``excluded`` range, each rounded up to 64 elements (tensor offsets are
    64-aligned, so the padding stays inside the tensor's slot), adjacent pieces merged, and while
    more than ``max_ranges`` remain the two pieces with the smallest gap between them merged --
    never across a ``forbidden`` range (values that are already the global sum). None when that
    cannot get below ``max_ranges``."""
    ex = sorted(excluded)
    keep = []
    for n in layout.names:
        lo = layout.offsets[n]
        hi = lo + layout.numel(n)
        if any(a <= lo and hi <= b for a, b in ex):
            continue
        assert lo % 64 == 0, 'layout offsets are 64-aligned'
        keep.append([lo, min(total, (hi + 63) // 64 * 64)])
    keep.sort()
    out = []
    for lo, hi in keep:
        if out and lo <= out[-1][1]:
            out[-1][1] = max(out[-1][1], hi)
        else:
            out.append([lo, hi])
    while len(out) > max_ranges:
        ok = [j for j in range(len(out) - 1)
              if not any(out[j][1] < b and a < out[j + 1][0] for a, b in forbidden)]
        if not ok:
            return None
        i = min(ok, key=lambda j: out[j + 1][0] - out[j][1])
        out[i][1] = out[i + 1][1]
        del out[i + 1]
    return [tuple(r) for r in out]


class Learner:
    def __init__(self, network: Network, replay, config, ctx: Optional[DistContext] = None,
                 use_graph: Optional[bool] = None, ps_client=None, actor=None):
        self.net = network
        self.replay = replay
        self.config = config
        self.ctx = ctx or DistContext(device=network.device)
        self.device = network.device
        B = config.minibatch_size
        self.B = B
        self.idx = torch.zeros(B, dtype=torch.int32, device=self.device)
        self.weights = torch.ones(B, dtype=torch.float32, device=self.device)
        self.prio = torch.zeros(B, dtype=torch.float32, device=self.device)
        self.loss = torch.zeros(1, dtype=torch.float32, device=self.device)
        # (an async-PS worker all-reduces nothing: no xgmi transport and no start-up probe, whose
        # collectives the parameter server rank -- inside serve() -- would never join)
        # data parallelism over xgmi: the fc weight gradient travels as its factors (executor
        # lowrank_spec: all-gather of the fc input rows + dL/dh rows, ~14x fewer bytes than the
        # gradient at B=32); the all-reduce then covers only the rest of the flat buffer
        self.tau = min(1.0, float(config.target_update_tau))
        tfreq = self._target_freq()
        ex = network.executor
        if hasattr(ex, 'fold_head'):
            ex.fold_head = bool(int(getattr(config, 'fold_head', 1)))
        if hasattr(ex, 'chain_dgrad'):
            ex.chain_dgrad = int(getattr(config, 'chain_dgrad', 0))
        if hasattr(ex, 'fold_spin') and self.ctx.enabled and self.ctx.ranks_share_gpu():
            # several ranks on ONE GPU (rehearsal): no intra-launch spin waits besides the collectives'
            # own (bounded, co-residency-sized) ones -- a fold tail starved by another rank's spinning
            # blocks expired its waiters and zeroed their dH (round 6, W = 4 big-batch rehearsal)
            ex.fold_spin = False
        # the fc weight / bias gradient formed inside the fused optimizer launch from the fc input
        # rows and dH rows (executor.can_defer_fc): no fp32 fc gradient round trip through HBM.
        # Under DP only with the low-rank exchange (the rows are then every rank's)
        sg = not (ps_client is None and network.fuses_sigma_grads(tfreq))
        self._defer_fc = bool(ps_client is None and int(getattr(config, 'fuse_fc_wgrad', 1))
                              and network.fuses_update(tfreq) and hasattr(ex, 'can_defer_fc')
                              and ex.can_defer_fc(B, sg))
        lr = None
        if (self.ctx.enabled and ps_client is None and int(getattr(config, 'lowrank_dense', 1))
                and getattr(config, 'overlap_allreduce', True) and hasattr(ex, 'lowrank_spec')
                and getattr(config, 'allreduce_dtype', 'fp32') == 'fp32'):
            lr = ex.lowrank_spec(B, sigma_fused=network.fuses_sigma_grads(tfreq), fused_fc=self._defer_fc)
        # data parallelism, fused step: the conv / output-layer weight gradients run inside the update
        # launch as in one process, and its dependent update jobs sum them over the ranks in-launch (the
        # xgmi transport's exchange channel, optim_pack.h kModeDp): no all-reduce launch, no separate
        # weight-gradient launch. Needs the low-rank fc exchange (the fc gradient is then formed from
        # every rank's rows inside the same launch).
        fuse_wu = int(getattr(config, 'fuse_wgrad_update', 1))
        want_dpx = bool(lr is not None and self._defer_fc and fuse_wu and hasattr(ex, 'can_defer_wgrad')
                        and ex.can_defer_wgrad(B, sg) and config.allreduce in ('xgmi', 'auto'))
        nslots = sum(1 for it in ex.upd_items if it[20] < 0) if want_dpx else 0
        self.reducer = GradAllReducer(self.ctx, network.grad, config.grad_bucket_mb,
                                      'rccl' if ps_client is not None else config.allreduce, config.allreduce_dtype,
                                      gather_bytes=lr['gather_bytes'] if lr else 0, exchange_slots=nslots)
        self._lowrank = None
        self._ar_ranges = []
        if lr and self.reducer.in_graph and self.reducer.can_gather:
            W = self.ctx.world_size
            ranges = _reduce_ranges(network.layout, network.grad.numel(), lr['ranges'] + lr.get('skip', []),
                                    forbidden=lr['ranges'])
            # (Nature: one remaining range; dueling: two, one launch each in stream order)
            if ranges and all((hi - lo_) % (4 * W) == 0 for lo_, hi in ranges):
                self._lowrank = {'gather': self.reducer.xgmi.allgather2, 'gather_args': self.reducer.xgmi.gather_args,
                                 'world': W, 'rank': self.ctx.rank}
                self._ar_ranges = ranges
        if self.ctx.enabled and self._lowrank is None:
            self._defer_fc = False         # (an all-reduced fc gradient must exist in the flat buffer)
        # async PS over xgmi (--ps_lowrank): the fc gradient is pushed as its factors (the server forms
        # it in its fused optimizer launch); the plan is the server's too (same config, same net)
        self._ps_lowrank = None
        if ps_client is not None and hasattr(ps_client, 'lowrank'):
            # (decided in make_ps_client and checked against the server's plan on every rank)
            self._ps_lowrank = ps_client.lowrank
            if self._ps_lowrank is not None:
                assert self._defer_fc or ex.can_defer_fc(B, True), 'low-rank push needs the fused fc path'
                self._defer_fc = True
        # conv weight gradients as deterministic chunk-group partials summed inside the fused
        # optimizer launch (executor.can_det_wgrad): one process only (DP all-reduces the flat
        # gradient, whose conv range then must hold the sums)
        self._det_wgrad = bool(not self.ctx.enabled and ps_client is None and int(getattr(config, 'det_wgrad', 0))
                               and network.fuses_update(tfreq) and hasattr(ex, 'can_det_wgrad')
                               and ex.can_det_wgrad(B))
        # the grouped conv / output-layer weight gradients run in the leading blocks of the fused
        # update's first launch, beside the fc update (executor.can_defer_wgrad): one process, or data
        # parallelism with the in-launch exchange (above)
        dp_fused = bool(self.ctx.enabled and want_dpx and self._lowrank is not None
                        and getattr(self.reducer, 'can_exchange', False))
        self._defer_wgrad = bool(((not self.ctx.enabled and ps_client is None) or dp_fused) and self._defer_fc
                                 and not self._det_wgrad and fuse_wu
                                 and hasattr(ex, 'can_defer_wgrad') and ex.can_defer_wgrad(B, sg))
        self._dp_fused = dp_fused and self._defer_wgrad
        if self._dp_fused:
            self._ar_ranges = []           # (nothing left for an all-reduce launch)
        if hasattr(ex, 'dp_exchange'):
            ex.dp_exchange = self.reducer.xgmi if self._dp_fused else None
        self.train_steps = 0           # reference DQNAgent.training_steps (host-side mirror)
        if use_graph is None:
            use_graph = bool(config.hip_graph) and self.device.type == 'cuda'
        self.use_graph = use_graph
        self._graphs = None
        self._warm = 0
        self._noise_gen = None
        # --async_ps worker: gradients go to the rank-0 parameter server, which answers with
        # its current parameters (parallel/async_ps.py); no local optimizer step
        self.ps = ps_client
        # fused acting: a DeviceActor whose acting step runs inside this learner's launches
        # (one more trunk/fc instance + one head workgroup); its own step() is then not used
        self.actor = actor if (actor is not None and actor.can_fuse(self.B)) else None
        # data parallelism: all-reduce the dense-layer gradients (fc: ~95% of Nature-CNN's
        # bytes) while the conv backward runs, then the conv gradients (config.overlap_allreduce)
        self._tail = None
        # (xgmi without the low-rank exchange: no split -- its all-reduce runs in stream order
        # after the whole backward, see _kernel_allreduce)
        self._split = bool(self.ctx.enabled and ps_client is None and getattr(config, 'overlap_allreduce', True)
                           and (not self.reducer.in_graph or self._lowrank is not None))
        self._dense_hi = network.dense_range()[1] if self._split else 0
        self._presampled = False    # this step's minibatch was drawn by the last optimizer launch
        # sync DP + --disable_target_replication: rank 0's target is broadcast after each hard
        # sync; the host mirrors the device global_step to know when (one read, here)
        self._own_target = bool(self.ctx.enabled and ps_client is None and self.tau >= 1.0
                                and getattr(config, 'disable_target_replication', False))
        self._host_step = int(network.global_step) if self._own_target else 0
        self._xgmi_check_every = max(1, int(getattr(config, 'allreduce_check_steps', 1000)))
        self.defer_per_insert = True   # see _defer_per_insert (False: the acting launch inserts)

    # ------------------------------------------------------------ step body
    def _sample_and_grad(self):
        r = self.replay
        per = getattr(r, 'prioritized', False)
        beta = None
        if per:
            # annealed in the sampling kernel from the device global_step
            beta = (self.net.global_step, self.config.per_beta0, self.config.per_beta_steps)
        if (getattr(self.net.executor, 'consumes_slots', False) and getattr(r, 'frame_mode', False)
                and self.device.type == 'cuda'):
            # one launch: indices + scalars + frame-slot tables; conv1 reads the ring. Uniform
            # replay: usually no launch at all — the previous step's optimizer launch drew this
            # batch ('opt'), or the Nature trunk draws it ('trunk')
            mode = self._sample_mode()
            if mode == 'opt' and self._presampled:
                batch = r.slot_batch(self.B)
            else:
                batch = r.sample_slots(self.B, beta, defer=mode == 'trunk')
            self.idx = batch['idx']
        else:
            if per:
                r.sample_prioritized(self.B, beta, self.idx, self.weights)
            else:
                r.sample_indices(self.B, self.idx)
            batch = r.gather(self.idx)
            if per:
                batch['weights'] = self.weights
        self.net.begin_step_noise()
        acting = None
        if self.actor is not None:
            assert 'frames' in batch, 'fused acting needs the slot-batch sampler'
            acting = self.actor.fused_args(defer_per=self._defer_per_insert())
        # noisy nets: the fused optimizer derives dL/dsigma itself (not for async-PS pushes)
        sg = not (self.ps is None and self.net.fuses_sigma_grads(self._target_freq()))
        if self._split:
            loss, prio, self._tail = self.net.compute_grads(batch, acting=acting, split=True, sigma_grads=sg,
                                                            lowrank=self._lowrank, defer_fc=self._defer_fc,
                                                            det_wgrad=self._det_wgrad, defer_wgrad=self._defer_wgrad)
        else:
            loss, prio = self.net.compute_grads(batch, acting=acting, sigma_grads=sg, defer_fc=self._defer_fc,
                                                det_wgrad=self._det_wgrad, defer_wgrad=self._defer_wgrad)
        # keep references (static buffers under graph capture) instead of copies
        self.loss = loss.view(1)
        self.prio = prio.view(-1)

    def _sample_mode(self) -> str:
        """Where the uniform minibatch is drawn: 'opt' (an extra block of the previous step's
        optimizer launch), 'trunk' (the Nature trunk launch) or 'launch' (a sampler launch)."""
        r = self.replay
        fs = int(getattr(self.config, 'fuse_sampling', 2))
        if (fs >= 2 and self.ps is None and getattr(r, 'can_fuse_sampling', lambda B: False)(self.B)
                and getattr(self.net.executor, 'consumes_slots', False)
                and self.net.fuses_update(self._target_freq())):
            return 'opt'            # (prioritized too: priority update + sample in that block)
        if getattr(r, 'prioritized', False) or not getattr(r, 'can_defer_sampling', lambda: False)():
            return 'launch'
        if fs >= 1 and getattr(self.net.executor, 'fused_sampling', False):
            return 'trunk'
        return 'launch'

    def _defer_per_insert(self) -> bool:
        """Prioritized replay + fused acting + 'opt' sampling: the optimizer launch's sampler
        block enters the actors' new transitions into the sum-tree (max priority) in the same
        one-wave climb as this step's priorities, instead of a serial climb at the end of the
        acting workgroup (the head launch's critical path)."""
        return (self.defer_per_insert and self.actor is not None and getattr(self.replay, 'prioritized', False)
                and self.B + self.actor.E <= 64 and self._sample_mode() == 'opt')

    def _target_freq(self):
        """target_freq argument of apply_grads: the hard sync rides in the optimizer launch."""
        return self.config.target_update_freq if self.tau >= 1.0 else None

    def _apply(self):
        cfg = self.config
        hard = self.tau >= 1.0
        # hard target sync folded into the optimizer + repack launches when the backend can
        # (and, 'opt' sampling, the NEXT step's minibatch drawn by one extra block of it)
        nxt = None
        per = getattr(self.replay, 'prioritized', False)
        if self._sample_mode() == 'opt':
            nxt = self.replay.next_sample_spec(
                self.B, per=(self.idx, self.prio, self.net.global_step, cfg.per_eps, cfg.per_beta0,
                             cfg.per_beta_steps) if per else None,
                insert=self.actor.per_insert_spec() if per and self._defer_per_insert() else None)
        fused = self.net.apply_grads(self.reducer.scale, target_freq=self._target_freq(), next_sample=nxt)
        self._presampled = nxt is not None and fused
        if per and not self._presampled:
            self.replay.update_priorities(self.idx, self.prio, cfg.per_eps)
        # hard copy when global_step % target_update_freq == 0 (device predicate, no sync).
        # Under sync DP every rank's online params are bit-identical, so the local
        # copy equals the reference's PS-owned target (--disable_target_replication).
        if not hard:
            kernels.target_update(self.net.target.flat, self.net.online.flat, self.tau)
            self.net.sync_target_copy(self.tau)
        elif not fused:
            self.net.hard_target_update(self.net.global_step, cfg.target_update_freq)

    def _run_tail(self):
        if self._tail is not None:
            self._tail()

    def _overlapped_allreduce(self, tail_runner):
        """dense-range all-reduce || conv backward (tail_runner), then the remaining range."""
        total = self.net.grad.numel()
        if self._tail is None or self._dense_hi <= 0:
            tail_runner()
            self.reducer.allreduce()
            return
        with trace('allreduce.dense'):
            h1 = self.reducer.allreduce_range_async(0, self._dense_hi)
        tail_runner()
        with trace('allreduce.rest'):
            h2 = self.reducer.allreduce_range_async(self._dense_hi, total)
        self.reducer.wait_all([h1, h2])

    def _kernel_allreduce(self):
        """xgmi transport: the all-reduces are kernel launches (graph-capturable), in stream
        order after the conv backward: a fork / join inside a captured HIP graph costs ~25 us on
        this ROCm (scripts/probe_graph_concurrency.py: one side kernel 11 -> 36 us), more than the
        overlap saves (round 2 measured the dense range on a side stream beside the conv backward:
        slower)."""
        total = self.net.grad.numel()
        if self._dp_fused:
            # the fused update launch sums every other gradient over the ranks itself (its dependent
            # jobs' in-launch exchange) and forms the fc gradient from the all-gathered rows: no launch
            self._run_tail()
            return
        if self._lowrank is not None and self._tail is not None:
            # the fc weight gradient is already the global sum (formed from the all-gathered
            # factors on the tail's joined branch): reduce only the remaining ranges
            self._tail()
            if len(self._ar_ranges) == 1:
                self.reducer.allreduce_range(*self._ar_ranges[0], channel=0)
            else:                                    # every remaining piece in ONE launch
                self.reducer.xgmi.allreduce_ranges(self.net.grad, self._ar_ranges, channel=0)
            return
        self._run_tail()
        self.reducer.allreduce_range(0, total, channel=0)

    def _eager_step(self):
        self._sample_and_grad()
        if self.ps is not None:
            self._run_tail()
            self._ps_exchange()
            return
        if self.reducer.in_graph:
            self._kernel_allreduce()
        elif self._split:
            self._overlapped_allreduce(self._run_tail)
        else:
            self.reducer.allreduce()
        self._apply()

    @property
    def stop_requested(self) -> bool:
        """The async parameter server answered STOP (no more pushes are accepted)."""
        return self.ps is not None and self.ps.stopped

    def _ps_in_graph(self) -> bool:
        """The PS exchange (push / pull kernels with device-side sequence numbers) and the repack
        ride in the step's HIP graph: the xgmi transport with replicated targets."""
        return (self.ps is not None and getattr(self.ps, 'in_graph', False)
                and not bool(self.config.disable_target_replication))

    def _ps_fc_rows(self):
        """Low-rank push: the deferred fc gradient's factor rows (taken off the executor: no local
        optimizer step consumes them)."""
        if self._ps_lowrank is None:
            return None
        ex = self.net.executor
        fc, ex._fc_pending = ex._fc_pending, None
        assert fc is not None, 'low-rank push: compute_grads(defer_fc=True) left no fc rows'
        return fc[0], fc[1]

    def _ps_exchange_kernels(self):
        """The graph-capturable part of the exchange: push + pull launches, then the repack."""
        self.ps.exchange_kernels(self.net.grad, self.net.online.flat, self.net.global_step, self._ps_fc_rows())
        self.net._repack()

    def _ps_after_graph(self):
        """Host side of an in-graph exchange: the push count and the LOCAL target cadence
        (reference `dqn_agent.py:143,215-222`), eager after the replay (stream order)."""
        self.ps.pushes += 1
        due = self.tau >= 1.0 and (self.train_steps + 1) % max(1, self.config.target_update_freq) == 0
        if self.tau < 1.0:
            self.update_target_now(self.tau)
        elif due:
            self.update_target_now()

    def _ps_exchange(self):
        """Async-PS worker: push grads, pull the PS parameters, repack; target cadence on
        the LOCAL train-step count (reference `dqn_agent.py:143,215-222`). With
        --disable_target_replication the sync is a request to the PS, which owns the target
        and ships it back when it changed."""
        own = bool(self.config.disable_target_replication)
        due = self.tau >= 1.0 and (self.train_steps + 1) % max(1, self.config.target_update_freq) == 0
        with trace('ps.exchange'):
            kw = {'fc_rows': self._ps_fc_rows()} if self._ps_lowrank is not None else {}
            ok = self.ps.exchange(self.net.grad, self.net.online.flat, self.net.global_step,
                                  sync_target=own and due, target=self.net.target.flat if own else None, **kw)
        if not ok:
            return
        self.net._repack()
        if self.tau < 1.0:
            self.update_target_now(self.tau)
        elif own:
            if self.ps.target_updated and hasattr(self.net.executor, 'repack'):
                self.net.executor.repack(self.net.target.flat)
        elif due:
            self.update_target_now()

    def finish_ps(self):
        """--async_ps worker, end of training: with --ps_pipeline the local parameters are one PS
        answer behind; take the answer to the last push and repack, so end-of-run evaluation, metrics
        and state use the server's parameters (before ``ps.close()``)."""
        fl = getattr(self.ps, 'flush', None)
        if fl is not None and fl(self.net.online.flat, self.net.global_step):
            self.net._repack()

    def _broadcast_owned_target(self):
        """Sync DP + --disable_target_replication: rank 0 owns the target (reference: target
        variables on the PS, `network.py:226-231`); after each hard sync its copy is broadcast
        and every rank's packed target fragments are rebuilt from it."""
        self._host_step += 1
        f = max(1, int(self.config.target_update_freq))
        if self._own_target and self._host_step % f == 0:
            with trace('target.broadcast'):
                import torch.distributed as dist
                dist.broadcast(self.net.target.flat, src=0)
                if hasattr(self.net.executor, 'repack'):
                    self.net.executor.repack(self.net.target.flat)

    # ------------------------------------------------------------ graph
    def _capture(self):
        with quiet_capture():
            self._capture_graphs()

    def _capture_graphs(self):
        # (thread-local capture mode: other host threads of the process -- Ape-X inference, the
        # async-PS client -- keep launching and synchronising their own streams meanwhile)
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        g_pre, g_post = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            if self.ps is not None:
                # xgmi transport: the whole worker step (gradient, push, pull, repack) is ONE graph;
                # otherwise the post-exchange work is host-driven (eager)
                inside = self._ps_in_graph()
                with torch.cuda.graph(g_pre, stream=s, capture_error_mode=_CAPTURE_MODE):
                    self._sample_and_grad()
                    if inside:
                        self._run_tail()
                        self._ps_exchange_kernels()
                self._graphs = (g_pre,)
            elif self.ctx.enabled and self.reducer.in_graph:
                # the whole DP step: ONE graph
                with torch.cuda.graph(g_pre, stream=s, capture_error_mode=_CAPTURE_MODE):
                    self._sample_and_grad()
                    self._kernel_allreduce()
                    self._apply()
                self._graphs = (g_pre,)
            elif self.ctx.enabled:
                with torch.cuda.graph(g_pre, stream=s, capture_error_mode=_CAPTURE_MODE):
                    self._sample_and_grad()
                g_tail = None
                if self._split and self._tail is not None:
                    g_tail = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g_tail, stream=s, capture_error_mode=_CAPTURE_MODE):
                        self._tail()
                with torch.cuda.graph(g_post, stream=s, capture_error_mode=_CAPTURE_MODE):
                    self._apply()
                self._graphs = (g_pre, g_post, g_tail)
            else:
                with torch.cuda.graph(g_pre, stream=s, capture_error_mode=_CAPTURE_MODE):
                    self._sample_and_grad()
                    self._apply()
                self._graphs = (g_pre,)
        torch.cuda.current_stream(self.device).wait_stream(s)

    # ------------------------------------------------------------- public
    def can_step_many(self) -> bool:
        """Whether ``step_many(k)`` replays ONE graph of k step bodies: one process, or data
        parallelism whose collectives are in-graph kernels (xgmi). (Round 2 measured 8-step graphs
        3x slower than one-step graphs with 2 ranks sharing ONE GPU, profiles/
        r2_dp_multistep_graphs.md; with one GPU per rank the benchmark decides by a start-up
        probe.)"""
        return (self.ps is None and self.use_graph and self._graphs is not None
                and (not self.ctx.enabled or self.reducer.in_graph) and not self._own_target)

    def step_many(self, k: int) -> torch.Tensor:
        """k SGD steps with ONE host call when ``can_step_many()``: a graph holding k consecutive
        step bodies (host-light learner loops, e.g. Ape-X, whose Python thread shares the GIL
        with the inference service; the benchmark); otherwise k ``step()`` calls. A refused
        capture raises with the host-side step state as before the attempt."""
        k = int(k)
        if k <= 1 or not self.can_step_many():
            for _ in range(max(1, k)):
                self.step()
            return self.loss
        g = getattr(self, '_graph_many', None)
        if g is None or g[0] != k:
            torch.cuda.synchronize(self.device)
            s = torch.cuda.Stream(device=self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            gk = torch.cuda.CUDAGraph()
            # host-side state a step body advances (restored if the capture is refused midway)
            ex = self.net.executor
            saved = (self._presampled, getattr(self.net, '_noise_drawn', False), getattr(ex, '_fc_pending', None),
                     getattr(ex, '_parts_pending', None), getattr(ex, '_wg_pending', None))
            try:
                with quiet_capture(), torch.cuda.stream(s), \
                        torch.cuda.graph(gk, stream=s, capture_error_mode=_CAPTURE_MODE):
                    for _ in range(k):
                        self._sample_and_grad()
                        if self.ctx.enabled:
                            self._kernel_allreduce()
                        self._apply()
            except Exception:
                self._presampled = saved[0]
                self.net._noise_drawn = saved[1]
                if hasattr(ex, '_fc_pending'):
                    ex._fc_pending, ex._parts_pending, ex._wg_pending = saved[2], saved[3], saved[4]
                torch.cuda.current_stream(self.device).wait_stream(s)
                raise
            torch.cuda.current_stream(self.device).wait_stream(s)
            self._graph_many = g = (k, gk)
        with trace('learner.step_many'):
            g[1].replay()
        if (self.train_steps + k) // self._xgmi_check_every != self.train_steps // self._xgmi_check_every:
            self._device_checks()
        self.train_steps += k
        return self.loss

    def step(self) -> torch.Tensor:
        """One SGD step. Returns the (device) TD-loss tensor; no host sync."""
        with trace('learner.step'):
            return self._step()

    def _step(self) -> torch.Tensor:
        if not self.use_graph or (self._graphs is None and self._warm < 2):
            # eager path; on the GPU the first two steps also warm up the
            # allocator, kernels and RCCL communicators before capture
            self._eager_step()
            self._warm += 1
        else:
            if self._graphs is None:
                torch.cuda.synchronize(self.device)
                self._capture()      # records only; the replay below runs the step
            self._graphs[0].replay()
            if self.ps is not None:
                if self._ps_in_graph():
                    self._ps_after_graph()
                else:
                    self._ps_exchange()
            elif len(self._graphs) > 1:
                g_tail = self._graphs[2]
                if g_tail is not None:
                    self._overlapped_allreduce(g_tail.replay)
                else:
                    with trace('allreduce'):
                        self.reducer.allreduce()
                self._graphs[1].replay()
        if self._own_target:
            self._broadcast_owned_target()
        self.train_steps += 1
        if self.train_steps % self._xgmi_check_every == 0:
            self._device_checks()
        return self.loss

    def _device_checks(self):
        """Error words the in-graph kernels leave instead of hanging, read off the hot path (one
        host sync per ``allreduce_check_steps``): the xgmi kernel's timed-out peer wait (its
        gradient is then only partly reduced) and the fused optimizer's end-of-launch wait
        (optim.hip kErrFlag). Fails loudly so the supervisor stops the run and the chief keeps
        its last consistent checkpoint."""
        if self.reducer.xgmi is not None:
            self.reducer.check()
        # async PS over xgmi: a pull / push whose peer wait timed out left this worker's
        # parameters un-pulled (the kernel flags it instead of hanging)
        chk = getattr(self.ps, 'check', None)
        if chk is not None and not chk():
            raise RuntimeError('async parameter server: a peer wait timed out (server stalled or gone) '
                               'at step %d' % self.train_steps)
        t = getattr(self.net.optimizer, 'ticket', None)
        if t is not None and t.is_cuda and t.numel() > 2 and int(t[2].item()) != 0:
            raise RuntimeError('fused optimizer: an end-of-launch arrival wait gave up (step %d)' % self.train_steps)
        fe = getattr(self.net.executor, 'fold_errors', None)
        errs = fe() if fe is not None else []
        if errs:
            raise RuntimeError('folded head: a dH block\'s wait for its group\'s dQ expired (groups %s, step %d); '
                               'its dH tile was not written' % ([e & 0xffff for e in errs], self.train_steps))

    def update_target_now(self, tau: float = 1.0):
        """Unconditional target sync (reference `_update_target_network` at init, `dqn_agent.py:50`)."""
        kernels.target_update(self.net.target.flat, self.net.online.flat, tau)
        self.net.sync_target_copy(tau)
