"""GPU-resident actor: E synthetic Atari environments stepped on the device.

Per call, ``steps_per_call`` times: stack the E current states from the
frame ring -> one batched online forward -> `actor_step` kernel (eps-greedy
with the reference's decay-before-roll schedule, synthetic env step, frame
write, replay append, cursor advance). The whole call is captured once into
a HIP graph, so acting costs one graph launch next to the learner's.

Used by the benchmark and by Ape-X-style runs that want actor throughput
without CPU emulators (no ALE here). CPU actor processes feeding the replay
through shared-memory rings live in `actors/apex.py`.
"""
from __future__ import annotations

import torch

from ..utils.capture import quiet_capture
from ..ops import _ext
from ..replay.device import DeviceReplay
from ..utils.trace import trace


class DeviceActor:
    def __init__(self, network, replay: DeviceReplay, config, num_envs: int = 1, steps_per_call: int = 4,
                 seed: int = 0, episode_len: int = 2000, use_graph: bool = True):
        assert replay.frame_mode and replay.device.type == 'cuda'
        self.net, self.replay, self.cfg = network, replay, config
        self.E, self.steps = num_envs, steps_per_call
        dev = replay.device
        self.dev = dev
        k = replay.k
        H, W = replay.obs_shape
        self.ext = _ext.load(required=True)
        # start every env on a fresh random reset frame
        r = replay
        base = r._f_next
        slots = (torch.arange(num_envs, device=dev) + base) % r.num_frames
        r.frames[slots.long()] = torch.randint(0, 256, (num_envs, H, W), dtype=torch.uint8, device=dev)
        self.stacks = slots.view(-1, 1).repeat(1, k).to(torch.int32).contiguous()
        f_next = (base + num_envs) % r.num_frames
        r.cursor = torch.tensor([r._t_next, f_next, r._size], dtype=torch.int64, device=dev)
        r.device_writer = True
        self.eps = torch.tensor([config.init_random_action_prob, config.min_random_action_prob,
                                 (config.init_random_action_prob - config.min_random_action_prob)
                                 / max(1, config.random_action_explore_steps)], dtype=torch.float32, device=dev)
        self.rng = torch.tensor([seed & 0x7fffffff, 0], dtype=torch.int64, device=dev)
        self.ticket = torch.zeros(1, dtype=torch.int32, device=dev)
        self.frames_done = torch.zeros(1, dtype=torch.int64, device=dev)
        self.states = torch.zeros(num_envs, H, W, k, dtype=torch.uint8, device=dev)
        self.gamma = float(config.reward_discount)
        self.p_done = 1.0 / float(episode_len)
        self.use_graph = use_graph
        self._graph = None
        self._warm = 0

    def _actor_args(self):
        r = self.replay
        ptrs = [0] + [t.data_ptr() for t in (r.frames, self.stacks, r.cursor, r.size_dev, r.state_idx,
                                               r.next_idx, r.actions, r.rewards, r.dones, r.gammas, self.eps,
                                               self.rng, self.ticket, self.frames_done)]
        ints = [self.E, self.net.arch.num_actions, r.k, r.frames.shape[1] * r.frames.shape[2], r.capacity,
                r.num_frames]
        if r.prioritized:              # new transitions enter the sum-tree at the running max priority
            t = r.tree
            ints += [t.sum.data_ptr(), t.min.data_ptr(), t.max_p.data_ptr(), t.P, t.P.bit_length() - 1]
        return ptrs, ints, [self.gamma, self.p_done]

    def can_fuse(self, batch_size: int) -> bool:
        """One acting step per learner step that the learner's launches can carry."""
        ex = self.net.executor
        return (self.steps == 1 and self.E <= min(64, batch_size) and getattr(ex, 'consumes_slots', False)
                and hasattr(ex, 'supports_fused_acting') and ex.supports_fused_acting())

    def fused_args(self, defer_per: bool = False) -> dict:
        """Arguments of the fused acting step (executor.loss_and_grad(acting=...)).
        defer_per (prioritized replay): the acting launch does not insert the new transitions
        into the sum-tree; the learner's optimizer launch does (`per_insert_spec`)."""
        ptrs, ints, f = self._actor_args()
        if defer_per:
            ints = ints[:6]
        return {'stacks': self.stacks, 'ptrs': ptrs, 'ints': ints, 'f': f}

    def per_insert_spec(self) -> list:
        """[cursor ptr, E, capacity]: where this step's E new transitions end (the acting
        launch advances cursor[0] past them) -- `DeviceReplay.next_sample_spec(insert=...)`."""
        r = self.replay
        return [r.cursor.data_ptr(), self.E, r.capacity]

    def _one(self):
        r = self.replay
        ex = self.net.executor
        if getattr(ex, 'consumes_slots', False) and self.E <= 64:
            # 3 launches: fused trunk reads the frame ring through the actors' stacks; the
            # eps-greedy / env step / replay append run inside the head kernel
            ptrs, ints, f = self._actor_args()
            ex.act_fused(self.net.online.flat, r.frames, self.stacks, ptrs, ints, f, noise=self.net.noise)
            return
        self.ext.stack_states(r.frames, self.stacks, self.states)
        q = self.net.q_values(self.states).float().contiguous()
        self.ext.actor_step(q, r.frames, self.stacks, r.cursor, r.size_dev, r.state_idx, r.next_idx, r.actions,
                            r.rewards, r.dones, r.gammas, self.eps, self.rng, self.ticket, self.frames_done,
                            self.gamma, self.p_done)

    def _body(self):
        for _ in range(self.steps):
            self._one()

    def step(self):
        with trace('actor.step'):
            self._step()

    def _step(self):
        if not self.use_graph or self._warm < 2:
            self._body()
            self._warm += 1
            return
        if self._graph is None:
            torch.cuda.synchronize(self.dev)
            s = torch.cuda.Stream(device=self.dev)
            s.wait_stream(torch.cuda.current_stream(self.dev))
            g = torch.cuda.CUDAGraph()
            with torch.cuda.stream(s):
                with quiet_capture(), torch.cuda.graph(g, stream=s):
                    self._body()
            torch.cuda.current_stream(self.dev).wait_stream(s)
            self._graph = g
        self._graph.replay()

    @property
    def epsilon(self) -> float:
        return float(self.eps[0])

    @property
    def env_frames(self) -> int:
        return int(self.frames_done[0])
