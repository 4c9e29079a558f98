"""Ape-X style distributed acting: many CPU actor processes, one GPU learner.

Reference: one actor per worker process, acting inside the worker's own
episode loop with a batch-1 `session.run` per greedy action against the PS
parameters (`/root/reference/src/dqn_agent.py:72-107,155-189`).

MI355X-native design:
  * actors are plain numpy processes (no torch, no HIP): env step, C++ frame
    preprocessing, per-actor fixed epsilon eps_i = base^(1 + alpha*i/(N-1))
    (Ape-X), and — for greedy steps — a post into their inference MAILBOX;
  * the learner process answers all pending mailboxes with ONE batched
    forward on the GPU (``serve``) using the live online weights, so actors
    never hold stale parameter copies and nothing is broadcast;
  * transitions travel through a lock-free SPSC ring per actor in shared
    memory (csrc/host/spsc_ring.cpp); a native ingest thread (csrc/ingest_server.cpp)
    moves them into pinned staging and ships them as H2D copies on its own stream
    ordered against the learner stream with events (frames stored once, slot stacks
    per actor), so the learner's Python thread only replays learner graphs (without the
    native thread: ``drain`` on the learner thread, replay/device.py);
  * CPU budget under a container CFS quota smaller than the visible CPUs (``--apex_pace``,
    default 0.9): the actor processes stay unpinned and pace themselves so their CPU time
    together is <= 0.9 x (quota - 3), so the quota never throttles the learner / ingest /
    inference threads (measured, 256 actors on a 16-CPU quota: learner 8.4k SGD steps/s and
    67k env frames/s, vs 0.8k / 40k when the actors and the learner thread were pinned to
    quota-many CPU ids, `profiles/r3_apex_256actors_pacing.jsonl`); ``--apex_pace=0`` keeps
    the pinned layout with one reserved CPU each (``--apex_reserve_cpus``);
  * under data parallelism every rank runs its own pool into its own replay
    shard (sharded replay; gradients all-reduced as usual).

Shared memory is a file under /dev/shm mapped by every process (numpy.memmap),
which keeps Python's SharedMemory resource tracker out of the actor lifecycle.
"""
from __future__ import annotations

import dataclasses
import logging
import multiprocessing as mp
import os
import random
import sys
import time
import uuid
from collections import deque
from typing import Callable, List, Optional, Sequence

import numpy as np

from ..utils.capture import quiet_capture

log = logging.getLogger(__name__)

# transition record: 16-byte header + observation payload
HEADER = np.dtype([('kind', 'u1'), ('done', 'u1'), ('pad', 'u2'), ('action', '<i4'), ('reward', '<f4'),
                   ('ret', '<f4')])
KIND_RESET, KIND_STEP = 0, 1
assert HEADER.itemsize == 16


def apex_epsilons(n: int, base: float = 0.4, alpha: float = 7.0) -> List[float]:
    """Ape-X per-actor exploration rates eps_i = base^(1 + alpha * i / (n - 1))."""
    if n == 1:
        return [base]
    return [base ** (1.0 + alpha * i / (n - 1)) for i in range(n)]


@dataclasses.dataclass
class ActorSpec:
    index: int
    env_id: str
    seed: int
    eps: float
    frames_per_state: int
    frame_hw: Optional[Sequence[int]]       # (H, W) for image envs, None for vector envs
    obs_dim: int                            # vector envs: observation length
    max_steps_per_episode: int
    ring_path: str
    ring_offset: int
    ring_bytes: int
    mbox_path: str
    mbox_bytes: int
    num_actors: int
    record_bytes: int
    state_bytes: int
    reward_clip: float = 0.0
    max_frames: int = 0                     # stop after this many env steps (0 = until told)
    cpus: Optional[Sequence[int]] = None    # CPUs the actor process may run on (None: inherited)
    # CPU pacing (--apex_pace): this actor's share of one CPU (0 = unpaced). The actor sleeps
    # whenever its CPU time runs ahead of share x wall time, so all actors together stay under
    # the container's CFS quota while spread over every visible CPU (no pinning)
    cpu_share: float = 0.0


def _map(path: str, nbytes: int, create: bool = False) -> np.memmap:
    return np.memmap(path, dtype=np.uint8, mode='w+' if create else 'r+', shape=(nbytes,))


def actor_main(spec: ActorSpec):
    """Actor process body (spawned): numpy + ctypes only."""
    import os
    from .. import envs
    from ..native import load
    # optional lower CPU priority (DQN_ACTOR_NICE): measured with 256 actors on a 16-core share,
    # nice 10 cut both env frames (50.9k -> 44.1k/s) and learner steps (2.0k -> 1.6k/s), so 0
    nice = int(os.environ.get('DQN_ACTOR_NICE', '0'))
    if nice:
        try:
            os.nice(nice)
        except OSError:
            pass
    if spec.cpus:
        try:
            os.sched_setaffinity(0, set(spec.cpus))
        except (OSError, AttributeError):
            pass
    lib = load()
    ring_all = _map(spec.ring_path, spec.ring_offset + spec.ring_bytes)
    ring = ring_all[spec.ring_offset:spec.ring_offset + spec.ring_bytes]
    mbox = _map(spec.mbox_path, spec.mbox_bytes)
    env = envs.make(spec.env_id, seed=spec.seed)
    rng = random.Random(spec.seed)
    n_act = env.action_space.n
    k = spec.frames_per_state
    image = spec.frame_hw is not None
    rec = np.zeros(spec.record_bytes, dtype=np.uint8)
    hdr = rec[:HEADER.itemsize].view(HEADER)
    payload = rec[HEADER.itemsize:]
    if image:
        H, W = spec.frame_hw
        frame = np.empty((H, W), dtype=np.uint8)
        stack = np.zeros((H, W, k), dtype=np.uint8)

    def observe(obs):
        if image:
            lib.preprocess(obs, H, W, out=frame)
            payload[:] = frame.reshape(-1)
            return frame
        v = np.asarray(obs, dtype=np.float32).reshape(-1)
        payload[:] = v.view(np.uint8)
        return v

    def push():
        while lib.ring_push(ring, rec, 1) == 0:      # ring full: learner backpressure
            if lib.mbox_stopped(mbox):
                return False
            time.sleep(0.0005)
        return True

    frames = 0
    share = float(spec.cpu_share)
    cpu0, wall0 = time.process_time(), time.monotonic()

    def pace():
        # (every 8 env steps) sleep off CPU time used beyond share x wall time
        over = (time.process_time() - cpu0) / share - (time.monotonic() - wall0)
        if over > 0.0:
            time.sleep(min(over, 0.05))

    while not lib.mbox_stopped(mbox):
        obs = observe(env.reset())
        hdr['kind'], hdr['done'], hdr['action'], hdr['reward'], hdr['ret'] = KIND_RESET, 0, 0, 0.0, 0.0
        if not push():
            break
        if image:
            stack[:] = frame[:, :, None]               # first frame duplicated k times
            state = stack
        else:
            state = obs.copy()
        ret, steps, done = 0.0, 0, False
        while not done and steps < spec.max_steps_per_episode:
            if rng.random() < spec.eps:
                a = rng.randrange(n_act)
            else:
                a = lib.mbox_request(mbox, spec.index, np.ascontiguousarray(state))
                if a < 0:                             # stop requested while waiting
                    return
            obs, r, done, _ = env.step(a)
            ret += r
            steps += 1
            frames += 1
            if spec.reward_clip > 0:
                r = float(np.clip(r, -spec.reward_clip, spec.reward_clip))
            o = observe(obs)
            hdr['kind'], hdr['done'], hdr['action'], hdr['reward'] = KIND_STEP, int(done), a, r
            # episode return rides on the last record (for the learner's stats)
            hdr['ret'] = ret if (done or steps >= spec.max_steps_per_episode) else np.float32('nan')
            if not push():
                return
            if image:
                stack[:, :, :-1] = stack[:, :, 1:]
                stack[:, :, -1] = o
            else:
                state = o.copy()
            if spec.max_frames and frames >= spec.max_frames:
                return
            if share > 0.0 and (frames & 7) == 0:
                pace()


class ApexActorPool:
    """Learner-side owner of the actor processes, their rings and mailboxes."""

    def __init__(self, env_id: str, num_actors: int, frames_per_state: int, frame_hw: Optional[Sequence[int]],
                 obs_dim: int, num_actions: int, max_steps_per_episode: int, seed: int = 0,
                 eps_base: float = 0.4, eps_alpha: float = 7.0, ring_capacity: int = 1024,
                 reward_clip: float = 0.0, max_frames_per_actor: int = 0, shm_dir: str = '/dev/shm',
                 start_method: str = 'spawn', n_step: int = 1, gamma: float = 0.99):
        from ..native import load
        self.lib = load()
        self.n = int(num_actors)
        self.k = int(frames_per_state)
        self.frame_hw = tuple(frame_hw) if frame_hw is not None else None
        self.num_actions = num_actions
        obs_bytes = (self.frame_hw[0] * self.frame_hw[1]) if self.frame_hw else 4 * obs_dim
        self.obs_dim = obs_dim
        self.record_bytes = HEADER.itemsize + obs_bytes
        self.state_bytes = (obs_bytes * self.k) if self.frame_hw else obs_bytes
        self.ring_capacity = ring_capacity
        rb = self.lib.ring_bytes(ring_capacity, self.record_bytes)
        self.ring_stride = (rb + 4095) // 4096 * 4096
        tag = uuid.uuid4().hex[:12]
        if not os.path.isdir(shm_dir):
            shm_dir = '/tmp'
        self.ring_path = os.path.join(shm_dir, 'dqn_apex_rings_%s' % tag)
        self.mbox_path = os.path.join(shm_dir, 'dqn_apex_mbox_%s' % tag)
        self.rings = _map(self.ring_path, self.ring_stride * self.n, create=True)
        for i in range(self.n):
            self.lib.ring_init(self.rings[i * self.ring_stride:(i + 1) * self.ring_stride], ring_capacity,
                               self.record_bytes)
        self.mbox_bytes = self.lib.mbox_region_bytes(self.n, self.state_bytes)
        self.mbox = _map(self.mbox_path, self.mbox_bytes, create=True)
        self.lib.mbox_init(self.mbox, self.n, self.state_bytes)
        self.eps = apex_epsilons(self.n, eps_base, eps_alpha)
        self.specs = [ActorSpec(i, env_id, seed + 7919 * (i + 1), self.eps[i], self.k, self.frame_hw, obs_dim,
                                max_steps_per_episode, self.ring_path, i * self.ring_stride, rb, self.mbox_path,
                                self.mbox_bytes, self.n, self.record_bytes, self.state_bytes, reward_clip,
                                max_frames_per_actor)
                      for i in range(self.n)]
        self._ctx = mp.get_context(start_method)
        self.procs: List[mp.Process] = []
        # server buffers (pinned when a GPU learner asks for them: set_pinned)
        self._states = np.zeros((self.n, self.state_bytes), dtype=np.uint8)
        self._ids = np.zeros(self.n, dtype=np.int32)
        self._seq = np.zeros(self.n, dtype=np.uint64)
        self._acts = np.zeros(self.n, dtype=np.int32)
        self._pop = np.zeros((ring_capacity, self.record_bytes), dtype=np.uint8)
        self.n_step, self.gamma = int(n_step), float(gamma)
        self._nstep = None
        if self.n_step > 1:
            from ..replay.nstep import NStepAccumulator
            self._nstep = [NStepAccumulator(self.n_step, self.gamma) for _ in range(self.n)]
        self.frames = 0                      # env steps ingested
        self.episodes = 0
        self.returns: deque = deque(maxlen=100)
        self.served = 0                      # greedy actions answered
        # native drain's staging ship cadence (0: flush on every drain; ApexTrainer batches)
        self.flush_min, self.flush_max_delay = 0, 0.0
        self._closed = False

    # -------------------------------------------------------------- life
    def set_actor_cpus(self, cpus: Optional[Sequence[int]]):
        """Restrict the actor processes to these CPUs (before ``start``)."""
        for sp in self.specs:
            sp.cpus = tuple(cpus) if cpus else None

    def set_actor_pacing(self, total_cpus: float):
        """Unpinned actors whose CPU time together stays under ``total_cpus`` (before ``start``)."""
        for sp in self.specs:
            sp.cpus = None
            sp.cpu_share = max(1e-3, float(total_cpus) / max(1, self.n))

    def start(self):
        for s in self.specs:
            p = self._ctx.Process(target=actor_main, args=(s,), daemon=True, name='apex-actor-%d' % s.index)
            p.start()
            self.procs.append(p)
        return self

    def alive(self) -> int:
        return sum(p.is_alive() for p in self.procs)

    def kill_actors(self):
        """SIGKILL every actor process this pool started (fault injection: the actors of one
        rank die; published ring records stay valid, a half-written one is never published)."""
        for p in self.procs:            # exact processes we started
            if p.is_alive():
                p.kill()
        for p in self.procs:
            p.join(5.0)

    def stop(self, timeout: float = 10.0):
        if self._closed:
            return
        self.lib.mbox_set_stop(self.mbox, 1)
        t0 = time.time()
        for p in self.procs:
            p.join(max(0.1, timeout - (time.time() - t0)))
        for p in self.procs:            # exact processes we started, never a pattern
            if p.is_alive():
                p.terminate()
                p.join(2.0)
        self._closed = True
        for path in (self.ring_path, self.mbox_path):
            try:
                os.unlink(path)
            except FileNotFoundError:
                pass

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()

    # ----------------------------------------------------------- serving
    def pin_states(self, torch):
        """Collect mailbox states straight into page-locked memory (a GPU learner's H2D copy
        source, no staging copy or per-batch pinning); returns that torch tensor [n, bytes]."""
        t = torch.zeros((self.n, self.state_bytes), dtype=torch.uint8, pin_memory=True)
        self._states = t.numpy()
        return t

    def serve(self, q_fn: Callable[[np.ndarray], np.ndarray], max_batch: Optional[int] = None) -> int:
        """Answer every pending mailbox with ONE batched forward. q_fn maps a uint8/f32
        state batch [m, ...] to actions [m] (int). Returns m."""
        m = self.lib.mbox_collect(self.mbox, self.n, self.state_bytes, self._states, self._ids, self._seq,
                                  max_batch or self.n)
        if m == 0:
            return 0
        raw = self._states[:m]
        if self.frame_hw:
            batch = raw.reshape(m, self.frame_hw[0], self.frame_hw[1], self.k)
        else:
            batch = raw.view(np.float32).reshape(m, self.obs_dim)
        self._acts[:m] = np.asarray(q_fn(batch), dtype=np.int32).reshape(-1)[:m]
        self.lib.mbox_respond(self.mbox, self.state_bytes, self._ids, self._seq, self._acts, m)
        self.served += m
        return m

    # ------------------------------------------------------------ ingest
    def drain(self, replay, max_per_actor: Optional[int] = None) -> int:
        """Move every actor's pending transitions into the replay's staging (then flush).
        Image envs with a frame-stacked HBM replay: ONE native call per actor
        (DeviceReplay.ingest_ring -> csrc/host/apex_ingest.cpp) reads the ring in place and
        writes frames, slot stacks and n-step transitions straight into the pinned staging;
        otherwise (vector observations) the per-record path below."""
        if self.frame_hw is not None and hasattr(replay, 'ingest_ring') and replay.frame_mode \
                and not replay.device_writer:
            return self._drain_native(replay, max_per_actor)
        total = 0
        hsz = HEADER.itemsize
        cap = min(self.ring_capacity, max_per_actor or self.ring_capacity)
        for i in range(self.n):
            ring = self.rings[i * self.ring_stride:(i + 1) * self.ring_stride]
            m = self.lib.ring_pop(ring, self._pop, cap)
            if m == 0:
                continue
            hdrs = self._pop[:m, :hsz].copy().view(HEADER).reshape(m)
            for j in range(m):
                h = hdrs[j]
                body = self._pop[j, hsz:]
                obs = body.reshape(self.frame_hw) if self.frame_hw else body.view(np.float32)
                if h['kind'] == KIND_RESET:
                    replay.begin_episode(obs.copy(), actor=i)
                    if self._nstep is not None:
                        self._nstep[i].reset()
                    continue
                if self._nstep is not None:
                    replay.add_step_nstep(self._nstep[i], int(h['action']), float(h['reward']), obs.copy(),
                                          bool(h['done']), actor=i)
                else:
                    replay.add_step(int(h['action']), float(h['reward']), obs.copy(), bool(h['done']), actor=i,
                                    gamma_n=self.gamma)
                self.frames += 1
                if not np.isnan(h['ret']):
                    self.episodes += 1
                    self.returns.append(float(h['ret']))
            total += m
        if total:
            replay.flush()
        return total


    def _drain_native(self, replay, max_per_actor: Optional[int]) -> int:
        """Staging is shipped (H2D copies + PER insert) once ``flush_min`` transitions are
        staged or ``flush_max_delay`` seconds passed, not per drain: a flush orders the copy
        stream after the queued learner steps, so flushing every loop iteration would hold the
        host to the GPU and the learner to the drain cadence."""
        if getattr(self, '_astate', None) is None:
            words = replay.ingest_state_size(self.k, self.n_step)
            self._astate = np.zeros((self.n, words), dtype=np.int32)
            base = self.rings.ctypes.data
            self._ring_addrs = np.array([base + i * self.ring_stride for i in range(self.n)], dtype=np.int64)
            self._last_flush = time.time()
        total, frames, eps, rets = replay.ingest_rings(self.lib, self._ring_addrs, self._astate, self.n_step,
                                                       self.gamma, -1 if max_per_actor is None else int(max_per_actor))
        self.frames += frames
        self.episodes += eps
        self.returns.extend(rets)
        now = time.time()
        if replay.staged() and (replay.staged() >= self.flush_min or now - self._last_flush >= self.flush_max_delay):
            replay.flush()
            self._last_flush = now
        return total


class ApexTrainer:
    """One learner rank of Ape-X: actor pool + inference thread + replay ingest + learner.

    The learner keeps the reference's train cadence knob differently: actors run
    free, and the learner takes an SGD step whenever the replay holds enough data
    (Ape-X). ``actor_param_sync_freq`` > 0 makes the inference service act with a
    parameter snapshot refreshed every that many learner steps (Ape-X actors'
    periodic parameter pulls); 0 acts with the live online weights.
    """

    def __init__(self, network, replay, learner, pool: ApexActorPool, config, metrics=None):
        import threading
        import torch
        self.torch = torch
        self.net, self.replay, self.learner, self.pool = network, replay, learner, pool
        self.config = config
        self.metrics = metrics
        self.device = network.device
        self.sync_freq = int(config.actor_param_sync_freq)
        self._snap = None
        self._synced = 0                    # snapshot refreshes done (every sync_freq learner steps)
        if self.sync_freq > 0:
            self._snap = network.online.flat.clone()
            self._refresh_snapshot()
        # inference I/O: states collected into pinned memory, one async H2D copy into a
        # persistent device buffer, actions back through a pinned buffer (one event wait)
        self._pin_in = self._dev_in = self._pin_out = None
        if self.device.type == 'cuda':
            self._pin_in = pool.pin_states(torch)
            self._dev_in = torch.zeros(self._pin_in.shape, dtype=torch.uint8, device=self.device)
            self._pin_out = torch.zeros(pool.n, dtype=torch.int32, pin_memory=True)
            self._gout = torch.zeros(pool.n, dtype=torch.int32, device=self.device)
            lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, 'priority_range') else (0, -1)
            self._istream = torch.cuda.Stream(device=self.device, priority=min(lo, hi))
            self._done = torch.cuda.Event()
        self._graphs = {}                   # batch size -> captured inference graph
        self._graphs_off = not bool(getattr(config, 'apex_infer_graphs', True))
        self._stop = threading.Event()
        self._lock = threading.Lock()       # one forward at a time vs the snapshot refresh
        self._thread = threading.Thread(target=self._serve_loop, name='apex-inference', daemon=True)
        pool.flush_min, pool.flush_max_delay = 256, 0.005     # ship staging in batches (see _drain_native)
        if hasattr(replay, 'ensure_stage_sets'):
            replay.ensure_stage_sets(6)     # flushes never wait on in-flight learner steps
        self.drain_every_s = 0.003          # ring drain cadence of the learner loop (each drain
                                            # costs GIL round trips with the inference thread)
        self.graph_steps = max(1, int(getattr(config, 'apex_graph_steps', 4)))   # SGD steps per host call
        self.max_inflight = max(2, 16 // self.graph_steps)   # queued launches before the loop waits
        self.gil_switch_s = 0.0005          # GIL hand-over interval while running
        self.serve_gap_s = float(getattr(config, 'apex_serve_gap_us', 100)) * 1e-6
        self.native_serve = bool(getattr(config, 'apex_native_serve', 1))
        self.serve_calls = 0
        self.learn_t0 = None                # wall time / env frames when the learner took its first step
        self.learn_frames0 = 0
        self.native_ingest = bool(getattr(config, 'apex_native_ingest', 1))
        self.reserve_cpus = int(getattr(config, 'apex_reserve_cpus', 3))
        self.pace = float(getattr(config, 'apex_pace', 0.9))
        self._ingest = None                 # native ingest server (csrc/ingest_server.cpp)
        self._cpus = None                   # (learner, ingest, inference) CPUs when reserved
        self.loop_time = {'drain': 0.0, 'step': 0.0, 'iters': 0}   # main-loop wall split (bench)

    def _refresh_snapshot(self):
        with self.torch.no_grad():
            self._snap.copy_(self.net.online.flat)
            if hasattr(self.net.executor, 'repack'):
                self.net.executor.repack(self._snap)

    def _act_on(self, x):
        """Greedy actions of a device state batch with the live (or snapshot) online weights."""
        if self._snap is not None:
            q = self.net.executor.q_values(self._snap, x.contiguous())
        else:
            q = self.net.q_values(x)
        return q.argmax(1).to(self.torch.int32)

    def _infer_graph(self, m: int, shape, f32: bool):
        """HIP graph of the whole inference for batch size m (device state buffer -> actions
        buffer): one replay call instead of the executor's per-launch Python work, which the
        inference thread would otherwise spend holding the GIL the learner loop needs."""
        torch = self.torch
        g = self._graphs.get(m)
        if g is not None or self._graphs_off:
            return g
        d = self._dev_in[:m]
        x = d.view(torch.float32).view(shape) if f32 else d.view(shape)
        try:
            with torch.cuda.stream(self._istream):
                self._gout[:m].copy_(self._act_on(x))          # warm-up: workspaces, packed buffers
            self._istream.synchronize()
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream(device=self.device)
            s.wait_stream(self._istream)
            with quiet_capture(), torch.cuda.stream(s), torch.cuda.graph(g, stream=s, capture_error_mode='thread_local'):
                self._gout[:m].copy_(self._act_on(x))
            self._istream.wait_stream(s)
            self._graphs[m] = g
        except Exception as e:  # noqa: BLE001 - fall back to eager inference, once
            log.warning('Ape-X inference graphs disabled (%s); serving eagerly', e)
            self._graphs_off = True
            g = None
        return g

    def _q_actions(self, batch: np.ndarray) -> np.ndarray:
        torch = self.torch
        m = batch.shape[0]
        with self._lock, torch.no_grad():
            if self._pin_in is None:
                return self._act_on(torch.from_numpy(batch)).numpy()
            f32 = batch.dtype == np.float32
            g = self._infer_graph(m, batch.shape, f32)
            # own high-priority stream: acting overlaps the queued learner steps instead of
            # waiting behind them (it reads the online weights while an update may be writing
            # them: a mix of two consecutive steps' weights, as stale as Ape-X acting allows)
            with torch.cuda.stream(self._istream):
                # batch is a view of the pinned collect buffer: one async H2D copy
                self._dev_in[:m].copy_(self._pin_in[:m], non_blocking=True)
                if g is not None:
                    g.replay()
                else:
                    d = self._dev_in[:m]
                    self._gout[:m].copy_(self._act_on(d.view(torch.float32).view(batch.shape) if f32
                                                      else d.view(batch.shape)))
                self._pin_out[:m].copy_(self._gout[:m], non_blocking=True)
                self._done.record()
            self._done.synchronize()         # (the actors wait for these actions)
            return self._pin_out[:m].numpy()

    def _start_native_server(self) -> bool:
        """Serve the mailboxes from a C++ thread (csrc/infer_server.cpp) replaying per-bucket
        inference graphs: the Python thread (and its GIL traffic) is not needed at all."""
        ext = getattr(self.net.executor, 'ext', None)
        if (self.device.type != 'cuda' or ext is None or not hasattr(ext, 'InferServer') or self._graphs_off
                or not self.native_serve):
            return False
        pool = self.pool
        n = pool.n
        shape = (pool.frame_hw[0], pool.frame_hw[1], pool.k) if pool.frame_hw else (pool.obs_dim,)
        f32 = pool.frame_hw is None
        sizes = sorted({min(n, 1 << i) for i in range(n.bit_length() + 1)} | {n})
        with self.torch.no_grad():
            for m in sizes:
                if self._infer_graph(m, (m,) + shape, f32) is None:
                    return False
        srv = ext.InferServer(int(pool.mbox.ctypes.data), n, pool.state_bytes, self._pin_in.data_ptr(),
                              self._dev_in.data_ptr(), self._gout.data_ptr(), self._pin_out.data_ptr(),
                              self.device.index if self.device.index is not None else 0,
                              int(self.serve_gap_s * 1e6))
        for m in sizes:
            srv.set_graph(m, self._graphs[m].raw_cuda_graph_exec())
        if self._cpus is not None and hasattr(srv, 'set_cpu'):
            srv.set_cpu(self._cpus[2])
        srv.start()
        self._server = srv
        log.info('Ape-X inference: native server thread, graph buckets %s', sizes)
        return True

    def _stop_native_server(self):
        srv = getattr(self, '_server', None)
        if srv is not None:
            srv.stop()
            served, calls, err = srv.stats()
            self.pool.served += int(served)
            self.serve_calls += int(calls)
            if err:
                log.error('Ape-X native inference server failed: %s', err)
            self._server = None

    # ----------------------------------------------------------- native ingest
    def _plan_cpus(self):
        """Reserve one CPU each for the learner thread, the ingest thread and the inference
        thread out of this process's CPU budget (the allowed set capped by the container's CFS
        quota, utils/cpus.py; when it leaves the actors at least 4); the actor processes are
        restricted to the rest, so together they never outrun the quota."""
        from ..utils.cpus import cfs_quota_cpus, usable_cpus
        try:
            allowed = sorted(os.sched_getaffinity(0))
        except AttributeError:
            return
        cpus = usable_cpus()
        r = self.reserve_cpus
        q = cfs_quota_cpus()
        if self.pace > 0 and q is not None and q < len(allowed):
            # paced, unpinned actors: their CPU time together <= pace x (quota - reserved), spread
            # over every visible CPU; the learner / ingest / inference threads keep no pinning
            budget = self.pace * max(1.0, float(q - max(r, 0)))
            self.pool.set_actor_pacing(budget)
            log.info('Ape-X: %d paced actors, %.1f CPUs of a %d-CPU CFS quota over %d visible CPUs',
                     self.pool.n, budget, q, len(allowed))
            return
        if r <= 0 or len(cpus) < r + 4:
            if len(cpus) < len(allowed):      # no reservation, but stay within the quota
                self.pool.set_actor_cpus(cpus)
                log.info('Ape-X: %d actors on %d CPUs (CFS quota %s)', self.pool.n, len(cpus), cfs_quota_cpus())
            return
        res = cpus[:r] + [cpus[r - 1]] * (3 - r) if r < 3 else cpus[:3]
        self._cpus = (res[0], res[1], res[2])
        self.pool.set_actor_cpus(cpus[r:])
        try:
            os.sched_setaffinity(0, {self._cpus[0]})      # this (learner) thread; restored by run()
            self._cpus_prev = allowed
        except OSError:
            self._cpus = None
            return
        log.info('Ape-X CPUs: learner %d, ingest %d, inference %d; %d actors on %d CPUs (%d visible, CFS quota %s)',
                 self._cpus[0], self._cpus[1], self._cpus[2], self.pool.n, len(cpus) - r, len(allowed),
                 cfs_quota_cpus())

    def _start_native_ingest(self) -> bool:
        """Ring ingest + H2D shipping on a C++ thread (csrc/ingest_server.cpp): the replay's
        host cursors are handed to it until ``_stop_native_ingest``."""
        r, pool = self.replay, self.pool
        ext = getattr(self.net.executor, 'ext', None)
        if (not self.native_ingest or self.device.type != 'cuda' or ext is None or not hasattr(ext, 'IngestServer')
                or pool.frame_hw is None or not getattr(r, 'frame_mode', False) or r.device_writer):
            return False
        torch = self.torch
        assert r.staged() == 0, 'native ingest starts with empty host staging'
        words = r.ingest_state_size(pool.k, pool.n_step)
        self._ing_state = np.zeros((pool.n, words), dtype=np.int32)
        base = pool.rings.ctypes.data
        self._ing_rings = np.array([base + i * pool.ring_stride for i in range(pool.n)], dtype=np.int64)
        H, W = r.obs_shape
        dev = [r.frames.data_ptr(), r.state_idx.data_ptr(), r.next_idx.data_ptr(), r.actions.data_ptr(),
               r.rewards.data_ptr(), r.dones.data_ptr(), r.gammas.data_ptr(), r.size_dev.data_ptr()]
        per = ([r.tree.sum.data_ptr(), r.tree.min.data_ptr(), r.tree.max_p.data_ptr(), r.tree.P]
               if r.prioritized else [0, 0, 0, 0])
        cfg = [pool.k, pool.n_step, H * W, r.capacity, r.num_frames, 1024, 6, 256, 5000,
               self.device.index if self.device.index is not None else 0,
               self._cpus[1] if self._cpus is not None else -1]
        stream = torch.cuda.current_stream(self.device)
        torch.cuda.synchronize(self.device)
        self._ingest = ext.IngestServer(int(self._ing_rings.ctypes.data), pool.n, int(self._ing_state.ctypes.data),
                                        words, float(pool.gamma), dev, per, [r._f_next, r._t_next, r._size], cfg,
                                        int(stream.cuda_stream))
        self._ingest_stream = stream
        self._ing_seen = (0, 0)
        self._ingest.start()
        log.info('Ape-X ingest: native thread (%d rings -> %d-transition pinned staging sets)', pool.n, 1024)
        return True

    def _ingest_poll(self):
        """Fold the native ingest's counters into the pool's (frames, episodes, returns)."""
        consumed, frames, eps, flushes, size, err = self._ingest.stats()
        if err:
            raise RuntimeError('Ape-X native ingest failed: %s' % err)
        f0, e0 = self._ing_seen
        self.pool.frames += frames - f0
        self.pool.episodes += eps - e0
        self._ing_seen = (frames, eps)
        self.pool.returns.extend(self._ingest.pop_returns())
        return size

    def _stop_native_ingest(self):
        srv, self._ingest = self._ingest, None
        if srv is None:
            return
        srv.stop()
        f, t, sz = srv.cursors()
        self._ingest = srv
        try:
            self._ingest_poll()
        finally:
            self._ingest = None
        r = self.replay
        r._f_next, r._t_next, r._size = int(f), int(t), int(sz)
        r._reset_stage()

    def _serve_loop(self):
        from ..utils.trace import trace
        while not self._stop.is_set():
            with trace('apex.serve'):
                m = self.pool.serve(self._q_actions)
            if m:
                self.serve_calls += 1
            # (a non-empty serve is followed by a short gap as well: requests accumulate into
            # larger batches and the learner loop gets the GIL between serves)
            time.sleep(self.serve_gap_s if m else 0.0002)

    def run(self, max_train_steps: int = 0, max_seconds: float = 0.0, supervisor=None, log_every: float = 10.0):
        from ..utils.trace import trace
        cfg = self.config
        start = max(cfg.minibatch_size, cfg.replay_start_size)
        self._plan_cpus()
        self.pool.start()
        if not self._start_native_server():
            self._thread.start()
        native = self._start_native_ingest()
        t0 = last = time.time()
        steps_at_last = frames_at_last = 0
        # sync-DP Ape-X: every learner step is a collective, so local reasons to stop (time
        # budget, dead actors) become stop requests the ranks agree on (supervisor.py)
        coordinated = bool(getattr(supervisor, 'coordinated', False))
        ctx = supervisor.ctx if coordinated else None
        started = not coordinated
        if supervisor is not None and hasattr(supervisor, 'fault_hooks'):
            supervisor.fault_hooks['actors'] = self.pool.kill_actors

        def want_stop(reason):
            if not coordinated:
                return True
            supervisor.request_stop(reason)
            return False

        # The learner thread and the inference thread share the GIL: drain on a time cadence
        # (the native ingest handles any backlog in one call) instead of per SGD step, bound the
        # queued graph launches with events (waiting on one releases the GIL), and hand the GIL
        # over at a finer interval so greedy requests are not parked behind learner launches.
        torch = self.torch
        cuda = self.device.type == 'cuda'
        inflight = deque()
        switch = sys.getswitchinterval()
        sys.setswitchinterval(self.gil_switch_s)
        last_drain = 0.0
        try:
            size = 0
            while True:
                ta = time.perf_counter()
                if native:
                    if ta - last_drain >= 0.01 or size < start:      # counters only: the thread ingests
                        size = self._ingest_poll()
                        last_drain = ta
                elif ta - last_drain >= self.drain_every_s or self.replay.size() < start:
                    with trace('apex.drain'):
                        self.pool.drain(self.replay)
                    last_drain = ta
                if not native:
                    size = self.replay.size()
                tb = time.perf_counter()
                self.loop_time['drain'] += tb - ta
                self.loop_time['iters'] += 1
                ready = size >= start
                if not started:
                    # sync-DP: every step is a collective, so the ranks take their first step
                    # together, once every rank's replay shard holds `start` transitions (one
                    # control-plane max per pre-start iteration: the ranks' collective sequences
                    # stay matched, and no in-graph xgmi wait spins on a peer still filling)
                    # (a stop asked for before the first step -- signal, time budget, dead actors --
                    # rides in the same max: 2 = some rank wants to stop, every rank leaves together)
                    v = ctx.ctrl_allreduce_max(2 if supervisor.stop_requested() else (0 if ready else 1))
                    if v >= 2:
                        log.info('apex: stop agreed before the first SGD step')
                        break
                    started = ready = v == 0
                if ready:
                    if self.learn_t0 is None:
                        self.learn_t0, self.learn_frames0 = time.time(), self.pool.frames
                    if cuda and len(inflight) >= self.max_inflight:
                        inflight.popleft().synchronize()
                    self.learner.step_many(self.graph_steps)
                    if cuda:
                        ev = torch.cuda.Event()
                        ev.record()
                        inflight.append(ev)
                    self.loop_time['step'] += time.perf_counter() - tb
                    if self._snap is not None and self.learner.train_steps // self.sync_freq != self._synced:
                        self._synced = self.learner.train_steps // self.sync_freq
                        with self._lock:
                            self._refresh_snapshot()
                    if supervisor is not None:
                        supervisor.on_train_step(self.learner.train_steps)
                else:
                    time.sleep(0.001)
                now = time.time()
                if now - last >= log_every:
                    dt = now - last
                    sps = (self.learner.train_steps - steps_at_last) / dt
                    fps = (self.pool.frames - frames_at_last) / dt
                    mean = float(np.mean(self.pool.returns)) if self.pool.returns else 0.0
                    log.info('apex: %d actors alive, frames %d (%.0f/s), sgd steps %d (%.1f/s), episodes %d, '
                             'last-100 mean return %.2f, replay %d', self.pool.alive(), self.pool.frames, fps,
                             self.learner.train_steps, sps, self.pool.episodes, mean, size)
                    if self.metrics is not None:
                        self.metrics.write(kind='apex', frames=self.pool.frames, env_frames_per_sec=fps,
                                           training_steps=self.learner.train_steps, sgd_steps_per_sec=sps,
                                           episodes=self.pool.episodes, mean100=mean,
                                           replay_size=size, actors_alive=self.pool.alive())
                    last, steps_at_last, frames_at_last = now, self.learner.train_steps, self.pool.frames
                if max_train_steps and self.learner.train_steps >= max_train_steps:
                    break
                if max_seconds and now - t0 >= max_seconds and want_stop('Ape-X time budget'):
                    break
                if supervisor is not None and supervisor.should_stop():
                    log.warning('Received signal to stop. Exiting Ape-X loop.')
                    break
                if self.pool.alive() == 0 and self.pool.procs:
                    if native:
                        self._stop_native_ingest()          # (its final pass drains the rings)
                        native = False
                    self.pool.drain(self.replay)
                    self.replay.flush()
                    size = self.replay.size()
                    if size < start:
                        if coordinated:
                            # this rank can never step again, so it cannot reach the agreed stop
                            # either: fail loudly (the peers' next collective fails, no final save)
                            raise RuntimeError('rank %d: all Ape-X actors exited before the replay reached %d '
                                               'transitions; cannot take part in the synchronous steps'
                                               % (getattr(supervisor, 'rank', 0), start))
                        log.warning('all actors exited')
                        break
                    if want_stop('all actors exited'):
                        log.warning('all actors exited')
                        break
        finally:
            self.end_t = time.time()
            sys.setswitchinterval(switch)
            self._stop.set()
            if self._thread.is_alive():
                self._thread.join(5.0)
            self.pool.lib.mbox_set_stop(self.pool.mbox, 1)      # (releases actors and the native server)
            self._stop_native_server()
            self._stop_native_ingest()
            self.pool.stop()
            prev = getattr(self, '_cpus_prev', None)
            if prev:
                try:
                    os.sched_setaffinity(0, set(prev))
                except OSError:
                    pass
        return self
