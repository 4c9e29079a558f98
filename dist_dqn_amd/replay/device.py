"""HBM-resident experience replay.

The reference stores every transition as a Python tuple holding the full
stacked state AND the full stacked next state (`/root/reference/src/replay_memory.py:22-23`,
`/root/reference/src/dqn_agent.py:99`): 2 x 84x84x4 bytes per transition, 56 GB
at the Atari capacity of 1M, re-fed to the GPU through ``feed_dict`` every
step (3.6 MB of f32 per minibatch).

Here the replay is a set of device tensors:
  * ``frames``    uint8 [F, H, W]   — each observation frame stored ONCE;
  * ``state_idx`` int32 [C, k]      — frame slots forming the state stack
    (episode-start frames duplicated exactly like the reference FrameBuffer);
  * ``next_idx``  int32 [C]         — slot of the newest frame of s'
    (s' = state_idx[1:] + [next_idx]);
  * ``actions`` int32, ``rewards`` f32, ``dones`` f32, ``gammas`` f32 [C]
    (gammas = gamma^n of the stored n-step transition).
Vector observations (CartPole) are stored directly as f32 [C, D] twice.

Frame ring size F = 2C + k + 8: every transition writes one frame and at most
one reset frame, so a valid transition's frames are never overwritten.
1M transitions = 14 GB of frames — 5% of one MI355X's 288 GB HBM — so the
default capacity per GPU can be far larger than the reference's.

Writes are staged in pinned host memory and flushed as contiguous H2D copies
on a side stream; sampling (uniform without replacement, or prioritized
through the device sum-tree) and the gather that rebuilds the uint8 stacks
run as HIP kernels inside the captured learner step (no host sync).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from ..ops import kernels


class _StageSet:
    """Persistent host staging buffers (pinned when the replay is on the GPU), exposed
    both as torch tensors (copy sources) and as numpy views (cheap per-step writes)."""

    def __init__(self, rep: 'DeviceReplay', n: int):
        pin = rep.device.type == 'cuda'

        def buf(shape, dtype):
            t = torch.zeros(shape, dtype=dtype, pin_memory=pin)
            return t, t.numpy()

        if rep.frame_mode:
            H, W = rep.obs_shape
            # every transition writes one frame, a reset one more: <= 2 frames per transition
            self.t_frames, self.frames = buf((2 * n + rep.k + 8, H, W), torch.uint8)
            self.t_sidx, self.sidx = buf((n, rep.k), torch.int32)
            self.t_nidx, self.nidx = buf((n,), torch.int32)
        else:
            self.t_frames, self.frames = buf((0,), torch.uint8)
            D = int(np.prod(rep.obs_shape))
            self.t_obs, self.obs = buf((n, D), torch.float32)
            self.t_nobs, self.nobs = buf((n, D), torch.float32)
        self.t_act, self.act = buf((n,), torch.int32)
        self.t_rew, self.rew = buf((n,), torch.float32)
        self.t_done, self.done = buf((n,), torch.float32)
        self.t_gam, self.gam = buf((n,), torch.float32)
        self.nf = self.nt = 0
        self.event = None

    def record(self, stream):
        self.event = torch.cuda.Event()
        self.event.record(stream)

    def wait(self):
        if self.event is not None:
            self.event.synchronize()
            self.event = None


class DeviceReplay:
    def __init__(self, capacity: int, obs_shape: Sequence[int], frames_per_state: int = 1,
                 device='cpu', num_actors: int = 1, prioritized: bool = False,
                 alpha: float = 0.6, stage_size: int = 1024, seed: int = 0):
        self.capacity = int(capacity)
        self.device = torch.device(device)
        self.k = int(frames_per_state)
        self.obs_shape = tuple(int(s) for s in obs_shape)
        self.frame_mode = len(self.obs_shape) == 2
        C = self.capacity
        dev = self.device
        if self.frame_mode:
            H, W = self.obs_shape
            self.num_frames = 2 * C + self.k + 8
            self.frames = torch.zeros(self.num_frames, H, W, dtype=torch.uint8, device=dev)
            self.state_idx = torch.zeros(C, self.k, dtype=torch.int32, device=dev)
            self.next_idx = torch.zeros(C, dtype=torch.int32, device=dev)
        else:
            D = int(np.prod(self.obs_shape))
            self.obs = torch.zeros(C, D, dtype=torch.float32, device=dev)
            self.next_obs = torch.zeros(C, D, dtype=torch.float32, device=dev)
        self.actions = torch.zeros(C, dtype=torch.int32, device=dev)
        self.rewards = torch.zeros(C, dtype=torch.float32, device=dev)
        self.dones = torch.zeros(C, dtype=torch.float32, device=dev)
        self.gammas = torch.ones(C, dtype=torch.float32, device=dev)
        # size lives on the device so graph-captured sampling reads the live value
        self.size_dev = torch.zeros(1, dtype=torch.int32, device=dev)
        # RNG state for in-kernel Philox sampling: [seed, counter]
        self.rng_state = torch.tensor([seed & 0x7fffffff, 0], dtype=torch.int64, device=dev)
        self._size = 0
        self._t_next = 0          # next transition slot
        self._f_next = 0          # next frame slot
        self.num_actors = num_actors
        self._stacks: List[Optional[List[int]]] = [None] * num_actors
        self._last_obs: List[Optional[np.ndarray]] = [None] * num_actors
        self.prioritized = prioritized
        self.alpha = alpha
        if prioritized:
            from .sumtree import DeviceSumTree
            self.tree = DeviceSumTree(C, dev)
        self._pin = self.device.type == 'cuda'
        self._stage_size = stage_size
        self._copy_stream = torch.cuda.Stream(device=self.device) if self._pin else None
        # two persistent (pinned) staging sets: one fills while the other's H2D copies drain
        self._sets = [_StageSet(self, stage_size) for _ in range(2 if self._pin else 1)]
        self._cur = 0
        self._reset_stage()
        # device-side writers (DeviceActor) keep [t_next, f_next, size] on the GPU
        self.cursor = None
        self.device_writer = False

    # ----------------------------------------------------------- staging
    def _reset_stage(self):
        st = self._sets[self._cur]
        st.wait()                       # its previous H2D copies must be done before refilling
        st.nf = st.nt = 0
        self._st_frame_first = self._f_next
        self._st_trans_first = self._t_next

    @property
    def _stage(self) -> '_StageSet':
        return self._sets[self._cur]

    def ensure_stage_sets(self, n: int):
        """At least n pinned staging sets in the rotation (default 2): a set is refilled only
        after its H2D copies ran, and those are ordered after the learner work queued before
        its flush, so a producer that flushes while many learner steps are in flight (Ape-X)
        needs a deeper rotation to never wait on them."""
        if self._pin:
            while len(self._sets) < n:
                self._sets.insert(self._cur + 1, _StageSet(self, self._stage_size))

    def _alloc_frame(self, frame) -> int:
        # frame slots are handed out sequentially, so staged frames are one
        # contiguous (wrap-split) range starting at _st_frame_first
        st = self._stage
        if st.nf == st.frames.shape[0]:
            self.flush()
            st = self._stage
        st.frames[st.nf] = frame
        st.nf += 1
        slot = self._f_next
        self._f_next = (self._f_next + 1) % self.num_frames
        return slot

    def _stage_transition(self, state, nxt, action, reward, done, gamma_n):
        st = self._stage
        i = st.nt
        if self.frame_mode:
            st.sidx[i] = state
            st.nidx[i] = nxt
        else:
            st.obs[i] = state
            st.nobs[i] = nxt
        st.act[i], st.rew[i], st.done[i], st.gam[i] = action, reward, done, gamma_n
        st.nt = i + 1
        if st.nt == self._stage_size:
            self.flush()

    def staged(self) -> int:
        """Transitions written but not yet flushed to the device."""
        return self._stage.nt

    def size(self) -> int:
        if self.device_writer:
            return int(self.size_dev[0])
        return self._size

    def __len__(self):
        return self.size()

    def digest(self) -> str:
        """Content fingerprint of the stored transitions (actions + rewards of the filled slots;
        one device sync): tells two shards fed by different actors apart."""
        import hashlib
        n = min(self.size(), self.capacity)
        h = hashlib.sha1()
        h.update(self.actions[:n].cpu().numpy().tobytes())
        h.update(self.rewards[:n].cpu().numpy().tobytes())
        return h.hexdigest()[:16]

    # ------------------------------------------------------------- write API
    def begin_episode(self, obs, actor: int = 0):
        """Start an episode: first frame duplicated k times (reference FrameBuffer semantics)."""
        if self.frame_mode:
            slot = self._alloc_frame(obs)
            self._stacks[actor] = [slot] * self.k
        else:
            self._last_obs[actor] = np.asarray(obs, dtype=np.float32).reshape(-1)

    def add_step(self, action: int, reward: float, next_obs, done: bool, actor: int = 0,
                 gamma_n: float = 1.0):
        """Append one transition whose state is the actor's current stack."""
        if self.frame_mode:
            st = self._stacks[actor]
            assert st is not None, 'begin_episode() first'
            slot = self._alloc_frame(next_obs)
            self._stage_transition(st, slot, action, reward, done, gamma_n)
            self._stacks[actor] = st[1:] + [slot]
        else:
            o = self._last_obs[actor]
            n = np.asarray(next_obs, dtype=np.float32).reshape(-1)
            self._stage_transition(o, n, action, reward, done, gamma_n)
            self._last_obs[actor] = n

    def add_step_nstep(self, acc, action: int, reward: float, next_obs, done: bool, actor: int = 0):
        """add_step through an n-step accumulator (replay.nstep.NStepAccumulator) owned by
        the caller, one per actor: frame stacks stay slot lists, so an n-step transition
        costs no extra frame storage."""
        if self.frame_mode:
            st = self._stacks[actor]
            assert st is not None, 'begin_episode() first'
            slot = self.write_frame(next_obs)
            nxt = st[1:] + [slot]
            self._stacks[actor] = nxt
            for s, a, R, ns, d, g in acc.push(list(st), action, reward, nxt, done):
                self.add_transition(s, ns[-1], a, R, d, g)
        else:
            prev = self._last_obs[actor]
            cur = np.asarray(next_obs, dtype=np.float32).reshape(-1)
            self._last_obs[actor] = cur
            for s, a, R, ns, d, g in acc.push(prev, action, reward, cur, done):
                self._stage_transition(s, ns, a, R, d, g)

    def add_transition(self, state_slots, next_slot, action, reward, done, gamma_n=1.0):
        """Low-level add with explicit frame slots (n-step / Ape-X actors)."""
        self._stage_transition(state_slots, next_slot, action, reward, done, gamma_n)

    def write_frame(self, frame) -> int:
        return self._alloc_frame(frame)

    @staticmethod
    def ingest_state_size(k: int, nstep: int) -> int:
        """int32 words of one actor's native ingest state (stack + n-step window)."""
        return k + 1 + nstep * (k + 2)

    def ingest_rings(self, lib, rings: np.ndarray, states: np.ndarray, nstep: int, gamma: float, max_n: int = -1):
        """``ingest_ring`` over many actors' rings (int64 addresses, one state row each) in one
        native call per staging set. Returns (consumed, frames, episodes, returns)."""
        assert self.frame_mode and not self.device_writer, 'native ingest: frame-stacked host-fed replay'
        H, W = self.obs_shape
        if getattr(self, '_ingm', None) is None:
            self._ingm = (np.zeros(13, dtype=np.int64), np.zeros(6, dtype=np.int64), np.zeros(1024, dtype=np.float32))
        arg, out, rbuf = self._ingm
        consumed = frames = episodes = 0
        rets: List[float] = []
        first = 0
        while True:
            st = self._stage
            arg[:] = [st.frames.ctypes.data, st.frames.shape[0], st.nf, st.sidx.ctypes.data, st.nidx.ctypes.data,
                      st.act.ctypes.data, st.rew.ctypes.data, st.done.ctypes.data, st.gam.ctypes.data,
                      st.act.shape[0], st.nt, self._f_next, self.num_frames]
            lib.apex_ingest_many(rings, states, first, max_n, self.k, nstep, gamma, H * W, arg, rbuf, out)
            st.nf, st.nt, self._f_next = int(arg[2]), int(arg[10]), int(arg[11])
            consumed += int(out[0])
            frames += int(out[1])
            episodes += int(out[2])
            rets.extend(rbuf[:int(out[3])].tolist())
            if st.nt >= self._stage_size:
                self.flush()
            if not out[4]:
                break
            first = int(out[5])
            self.flush()                    # staging full: ship it, resume with that actor
        return consumed, frames, episodes, rets

    def ingest_ring(self, lib, ring, actor_state: np.ndarray, nstep: int, gamma: float, max_n: int = -1):
        """Ape-X: move one actor's pending ring records straight into the pinned staging with the
        native ingest (csrc/host/apex_ingest.cpp: frames, slot stacks and the n-step fold, the
        same transitions begin_episode / add_step(_nstep) would stage), flushing whenever the
        staging fills. ``actor_state``: that actor's int32 ingest state (``ingest_state_size``).
        Returns (records consumed, env frames, episodes ended, their returns (the first 256 per
        native call))."""
        assert self.frame_mode and not self.device_writer, 'native ingest: frame-stacked host-fed replay'
        H, W = self.obs_shape
        if getattr(self, '_ing', None) is None:
            self._ing = (np.zeros(13, dtype=np.int64), np.zeros(5, dtype=np.int64), np.zeros(256, dtype=np.float32))
        arg, out, rbuf = self._ing
        consumed = frames = episodes = 0
        rets: List[float] = []
        while max_n < 0 or consumed < max_n:
            st = self._stage
            arg[:] = [st.frames.ctypes.data, st.frames.shape[0], st.nf, st.sidx.ctypes.data, st.nidx.ctypes.data,
                      st.act.ctypes.data, st.rew.ctypes.data, st.done.ctypes.data, st.gam.ctypes.data,
                      st.act.shape[0], st.nt, self._f_next, self.num_frames]
            lib.apex_ingest(ring, -1 if max_n < 0 else max_n - consumed, actor_state, self.k, nstep, gamma, H * W,
                            arg, rbuf, out)
            st.nf, st.nt, self._f_next = int(arg[2]), int(arg[10]), int(arg[11])
            consumed += int(out[0])
            frames += int(out[1])
            episodes += int(out[2])
            rets.extend(rbuf[:int(out[3])].tolist())
            if st.nt >= self._stage_size:
                self.flush()
            if not out[4]:
                break
            self.flush()                    # staging full: ship it and continue with the next set
        return consumed, frames, episodes, rets

    def flush(self):
        """Copy staged frames/transitions into the device ring (contiguous, wrap-split)
        as async H2D copies on the side stream, then switch staging sets."""
        st = self._stage
        assert not self.device_writer or not (st.nf or st.nt), \
            'a replay is fed either by host staging or by device actors, not both'
        if not st.nf and not st.nt:
            return
        cs = self._copy_stream
        if cs is not None:
            cs.wait_stream(torch.cuda.current_stream(self.device))   # ring slots may still be read
        if st.nf:
            self._ring_copy(self.frames, self._st_frame_first, st.t_frames[:st.nf])
        n = st.nt
        if n:
            first = self._st_trans_first
            if self.frame_mode:
                self._ring_copy(self.state_idx, first, st.t_sidx[:n])
                self._ring_copy(self.next_idx, first, st.t_nidx[:n])
            else:
                self._ring_copy(self.obs, first, st.t_obs[:n])
                self._ring_copy(self.next_obs, first, st.t_nobs[:n])
            self._ring_copy(self.actions, first, st.t_act[:n])
            self._ring_copy(self.rewards, first, st.t_rew[:n])
            self._ring_copy(self.dones, first, st.t_done[:n])
            self._ring_copy(self.gammas, first, st.t_gam[:n])
            self._t_next = (first + n) % self.capacity
            self._size = min(self.capacity, self._size + n)
            if self.prioritized:
                idx = (torch.arange(n, dtype=torch.int64) + first) % self.capacity
                self.tree.set_max_priority(idx.to(self.device, torch.int32))
        if cs is not None:
            st.record(cs)
        self._sync_copies()
        self.size_dev.fill_(self._size)
        self._cur = (self._cur + 1) % len(self._sets)
        self._reset_stage()

    def _ring_copy(self, dst: torch.Tensor, first: int, src: torch.Tensor):
        cap = dst.shape[0]
        n = src.shape[0]
        end = first + n
        if end <= cap:
            self._copy(dst[first:end], src)
        else:
            k = cap - first
            self._copy(dst[first:], src[:k])
            self._copy(dst[:end - cap], src[k:])

    def _copy(self, dst, src):
        if self._copy_stream is not None:
            with torch.cuda.stream(self._copy_stream):
                dst.copy_(src, non_blocking=True)
        else:
            dst.copy_(src)

    def _sync_copies(self):
        if self._copy_stream is not None:
            torch.cuda.current_stream(self.device).wait_stream(self._copy_stream)

    # ------------------------------------------------------------- read API
    def sample_indices(self, batch_size: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Uniform sample WITHOUT replacement (reference: random.sample), device-side."""
        if out is None:
            out = torch.empty(batch_size, dtype=torch.int32, device=self.device)
        kernels.replay_sample_uniform(self.size_dev, self.rng_state, out)
        return out

    def sample_prioritized(self, batch_size: int, beta: torch.Tensor, idx_out=None, w_out=None):
        if idx_out is None:
            idx_out = torch.empty(batch_size, dtype=torch.int32, device=self.device)
        if w_out is None:
            w_out = torch.empty(batch_size, dtype=torch.float32, device=self.device)
        self.tree.sample(self.rng_state, self.size_dev, beta, idx_out, w_out)
        return idx_out, w_out

    def sample_slots(self, batch_size: int, beta: Optional[torch.Tensor] = None,
                     defer: bool = False) -> Dict[str, torch.Tensor]:
        """GPU fast path: ONE sampling launch returns indices, per-sample scalars and the
        frame-slot tables of s and s' ([B, k] int32) — executors that read the frame ring
        directly (the HIP executor's conv1) never materialise the uint8 stacks.

        defer=True (uniform, k = 4): NO launch; the returned buffers are filled by the
        consumer's first kernel instead (the Nature trunk draws the batch itself, see
        csrc/kernels/sample_dev.h): ``out['sample_spec']`` holds the pointers it needs."""
        assert self.frame_mode and self.device.type == 'cuda'
        B = batch_size
        buf = self._slot_buffers(B)
        if defer and self.can_defer_sampling():
            if getattr(self, '_sample_ticket', None) is None:
                self._sample_ticket = torch.zeros(1, dtype=torch.int32, device=self.device)
            out = {k: buf[k] for k in ('idx', 'actions', 'rewards', 'dones', 'gammas', 'state_slots', 'next_slots')}
            out['frames'] = self.frames
            out['sample_spec'] = [t.data_ptr() for t in (
                self.size_dev, self.rng_state, self._sample_ticket, self.state_idx, self.next_idx, self.actions,
                self.rewards, self.dones, self.gammas, buf['idx'], buf['actions'], buf['rewards'], buf['dones'],
                buf['gammas'], buf['state_slots'], buf['next_slots'])]
            return out
        so = [self.state_idx, self.next_idx, self.actions, self.rewards, self.dones, self.gammas,
              buf['actions'], buf['rewards'], buf['dones'], buf['gammas'], buf['state_slots'], buf['next_slots']]
        if self.prioritized:
            assert beta is not None
            kernels.sumtree_sample(self.tree, self.rng_state, self.size_dev, beta, buf['idx'], buf['weights'], so)
        else:
            kernels.replay_sample_uniform(self.size_dev, self.rng_state, buf['idx'], so)
        out = {k: buf[k] for k in ('idx', 'actions', 'rewards', 'dones', 'gammas', 'state_slots', 'next_slots')}
        out['frames'] = self.frames
        if self.prioritized:
            out['weights'] = buf['weights']
        return out

    def _slot_buffers(self, B: int) -> dict:
        if not hasattr(self, '_slot_bufs'):
            self._slot_bufs = {}
        buf = self._slot_bufs.get(B)
        if buf is None:
            dev = self.device
            i32 = dict(dtype=torch.int32, device=dev)
            f32 = dict(dtype=torch.float32, device=dev)
            buf = {'idx': torch.zeros(B, **i32), 'weights': torch.ones(B, **f32),
                   'actions': torch.zeros(B, **i32), 'rewards': torch.zeros(B, **f32),
                   'dones': torch.zeros(B, **f32), 'gammas': torch.zeros(B, **f32),
                   'state_slots': torch.zeros(B, self.k, **i32), 'next_slots': torch.zeros(B, self.k, **i32)}
            self._slot_bufs[B] = buf
        return buf

    def slot_batch(self, B: int) -> Dict[str, torch.Tensor]:
        """The minibatch buffers as they are (no launch): a batch some earlier kernel drew
        (the optimizer launch's sampler block, see ``next_sample_spec``)."""
        buf = self._slot_buffers(B)
        out = {k: buf[k] for k in ('idx', 'actions', 'rewards', 'dones', 'gammas', 'state_slots', 'next_slots')}
        out['frames'] = self.frames
        if self.prioritized:
            out['weights'] = buf['weights']
        return out

    def can_fuse_sampling(self, B: int) -> bool:
        """The next minibatch can be drawn by an extra block of the optimizer launch."""
        ok = self.frame_mode and self.device.type == 'cuda' and self.k == 4 and 1 <= B <= 512
        return ok and (not self.prioritized or B <= 64)

    def next_sample_spec(self, B: int, per=None, insert=None) -> dict:
        """Arguments of the optimizer launch's sampler block (csrc/kernels/optim.hip): it draws
        the NEXT minibatch into ``slot_batch(B)``'s buffers. per (prioritized replay):
        (upd_idx, upd_td, global_step, per_eps, beta0, beta_steps) — the block first writes
        this step's priorities |td| of upd_idx into the sum-tree, then samples from it.
        insert (prioritized, fused acting): [cursor ptr, E, capacity] of the device actors whose
        E new transitions this step's launches appended -- the same block enters them into the
        tree at max priority in the same climb, before this step's priorities (the acting
        launch then skips its own insertion; `DeviceActor.fused_args(defer_per=True)`)."""
        buf = self._slot_buffers(B)
        if not self.prioritized:
            if getattr(self, '_sample_ticket', None) is None:
                self._sample_ticket = torch.zeros(1, dtype=torch.int32, device=self.device)
            return {'kind': 'uniform', 'B': B, 'spec': [t.data_ptr() for t in (
                self.size_dev, self.rng_state, self._sample_ticket, self.state_idx, self.next_idx, self.actions,
                self.rewards, self.dones, self.gammas, buf['idx'], buf['actions'], buf['rewards'], buf['dones'],
                buf['gammas'], buf['state_slots'], buf['next_slots'])]}
        upd_idx, upd_td, step, eps, beta0, beta_steps = per
        t = self.tree
        levels = t.P.bit_length() - 1
        ptr = lambda x: x.data_ptr()
        p = [ptr(t.sum), ptr(t.min), ptr(t.max_p), t.P, levels, ptr(upd_idx), ptr(upd_td), ptr(self.rng_state),
             ptr(self.size_dev), ptr(step), ptr(buf['idx']), ptr(buf['weights']), ptr(self.state_idx),
             ptr(self.next_idx), ptr(self.actions), ptr(self.rewards), ptr(self.dones), ptr(self.gammas),
             ptr(buf['actions']), ptr(buf['rewards']), ptr(buf['dones']), ptr(buf['gammas']),
             ptr(buf['state_slots']), ptr(buf['next_slots']), B]
        if insert is not None:
            assert B + int(insert[1]) <= 64, 'batch + inserted transitions must fit one wave'
            p += [int(v) for v in insert]
        return {'kind': 'per', 'p': p, 'f': [float(self.alpha), float(eps), float(beta0), float(max(1, beta_steps))]}

    def can_defer_sampling(self) -> bool:
        """Uniform frame-stacked (k = 4) GPU replay: a consumer kernel may draw the batch."""
        return self.frame_mode and self.device.type == 'cuda' and not self.prioritized and self.k == 4

    def update_priorities(self, idx: torch.Tensor, td_abs: torch.Tensor, eps: float = 1e-6):
        self.tree.update(idx, td_abs, self.alpha, eps)

    def gather(self, idx: torch.Tensor) -> Dict[str, torch.Tensor]:
        """Materialise a minibatch: states/next_states (uint8 NHWC stacks or f32 vectors).

        On the GPU the frame stacks and the per-sample columns come from ONE
        gather launch into persistent per-batch-size buffers (graph-safe)."""
        if self.frame_mode and self.device.type == 'cuda':
            B = idx.numel()
            buf = self._gather_bufs.get(B) if hasattr(self, '_gather_bufs') else None
            if buf is None:
                H, W = self.obs_shape
                dev = self.device
                buf = {'states': torch.empty(B, H, W, self.k, dtype=torch.uint8, device=dev),
                       'next_states': torch.empty(B, H, W, self.k, dtype=torch.uint8, device=dev),
                       'actions': torch.empty(B, dtype=torch.int32, device=dev),
                       'rewards': torch.empty(B, dtype=torch.float32, device=dev),
                       'dones': torch.empty(B, dtype=torch.float32, device=dev),
                       'gammas': torch.empty(B, dtype=torch.float32, device=dev)}
                if not hasattr(self, '_gather_bufs'):
                    self._gather_bufs = {}
                self._gather_bufs[B] = buf
            kernels.replay_gather_frames(
                self.frames, self.state_idx, self.next_idx, idx, (buf['states'], buf['next_states']),
                [self.actions, self.rewards, self.dones, self.gammas,
                 buf['actions'], buf['rewards'], buf['dones'], buf['gammas']])
            return dict(buf)
        out = {
            'actions': self.actions.index_select(0, idx.long()),
            'rewards': self.rewards.index_select(0, idx.long()),
            'dones': self.dones.index_select(0, idx.long()),
            'gammas': self.gammas.index_select(0, idx.long()),
        }
        if self.frame_mode:
            out['states'], out['next_states'] = kernels.replay_gather_frames(
                self.frames, self.state_idx, self.next_idx, idx)
        else:
            out['states'] = self.obs.index_select(0, idx.long())
            out['next_states'] = self.next_obs.index_select(0, idx.long())
        return out

    def fill_synthetic(self, n: int, num_actions: int, seed: int = 0, episode_len: int = 500):
        """Fill n transitions with synthetic random frames/rewards directly on the device
        (benchmarks: "synthetic frames"). Episodes of ``episode_len`` steps with the reference's
        duplicated first frame; frames are uniform random bytes."""
        n = min(n, self.capacity)
        g = torch.Generator(device=self.device).manual_seed(seed)
        if self.frame_mode:
            nf = n + n // episode_len + self.k + 1
            self.frames[:nf].random_(0, 256, generator=g)
            t = torch.arange(n, device=self.device)
            ep = t // episode_len
            pos = t - ep * episode_len
            first = ep * (episode_len + 1)                   # frame slot of each episode's reset frame
            cur = first + pos                                # newest frame of state t
            ks = torch.arange(self.k, device=self.device)
            slots = cur.view(-1, 1) - (self.k - 1 - ks).view(1, -1)
            slots = torch.maximum(slots, first.view(-1, 1))  # duplicate the episode's first frame
            self.state_idx[:n] = slots.to(torch.int32)
            self.next_idx[:n] = (cur + 1).to(torch.int32)
            self._f_next = int(nf) % self.num_frames
        else:
            self.obs[:n].normal_(generator=g)
            self.next_obs[:n].normal_(generator=g)
        self.actions[:n].random_(0, num_actions, generator=g)
        self.rewards[:n] = (torch.rand(n, device=self.device, generator=g) < 0.02).float()
        self.dones[:n] = 0.0
        if self.frame_mode:
            self.dones[:n][(torch.arange(n, device=self.device) % episode_len) == episode_len - 1] = 1.0
        self.gammas[:n] = 0.99
        self._size = n
        self._t_next = n % self.capacity
        self.size_dev.fill_(n)
        if self.prioritized:
            self.tree.set_max_priority(torch.arange(n, dtype=torch.int32, device=self.device))

    def nbytes(self) -> int:
        ts = [self.actions, self.rewards, self.dones, self.gammas]
        ts += [self.frames, self.state_idx, self.next_idx] if self.frame_mode else [self.obs, self.next_obs]
        return sum(t.numel() * t.element_size() for t in ts)
