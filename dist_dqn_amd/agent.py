"""DQNAgent — the reference's RL control loop with the same public API
(`/root/reference/src/dqn_agent.py:13-285`):

  DQNAgent(env, network, session, replay_memory, config, enable_summary=True)
  .train(num_episodes, max_steps_per_episode, supervisor=None)
  .train_episode(max_steps) -> (total_reward, steps)
  DQNAgent.get_input_shape(env, config)

Semantics kept exactly: epsilon decays linearly BEFORE the
dice roll on every ``_pick_action`` call (never during prefill); train once
every ``update_freq`` in-episode steps, skipped while replay < minibatch;
target copy at init and whenever ``training_steps % target_update_freq == 0``;
unclipped rewards (``--reward_clip`` is an opt-in extension); an episode cut
at ``max_steps_per_episode`` is not stored as terminal.

What changed is where the work runs: ``session`` is a `Learner` (device-
resident, HIP-graph-captured SGD step) instead of a ``tf.Session``; the
replay may be the reference host `ReplayMemory` (CPU) or the HBM
`DeviceReplay`; action selection is one batched forward on the device.
"""
from __future__ import annotations

import logging
import random
import time
from functools import partial
from typing import Optional

import numpy as np
import torch

from . import utils
from .frame_buffer import FrameBuffer
from .replay.device import DeviceReplay
from .replay.host import ReplayMemory
from .replay.nstep import NStepAccumulator
from .stats import RateMeter, Stats

log = logging.getLogger(__name__)


class DQNAgent:
    # Reward penalty on failure for each environment (reference: empty)
    FAILURE_PENALTY = {}

    def __init__(self, env, network, session, replay_memory, config, enable_summary=True,
                 summary_writer=None, metrics=None, monitor=None, rng: Optional[random.Random] = None):
        self.env = env
        self.network = network
        self.replay_memory = replay_memory
        self.config = config
        self.rng = rng or random.Random(config.seed)
        self.training_steps = 0
        self.stats = Stats()
        self.random_action_prob = config.init_random_action_prob
        self.random_action_prob_decay = utils.decay_per_step(
            init_val=config.init_random_action_prob,
            min_val=config.min_random_action_prob,
            steps=config.random_action_explore_steps)
        if session is None:
            from .learner import Learner
            session = Learner(network, replay_memory, config) if isinstance(replay_memory, DeviceReplay) else None
        self.session = session
        self.summary_writer = None
        if enable_summary:
            if summary_writer is None:
                from .utils.metrics import SummaryWriter
                summary_writer = SummaryWriter(config.logdir)
            self.summary_writer = summary_writer
        self.metrics = metrics
        self.monitor = monitor
        self._supervisor = None
        self.sgd_meter = RateMeter()
        self.frame_meter = RateMeter()
        self.frame_buffer = FrameBuffer(config.frames_per_state, self._get_frame_resizer(env, config))
        self._device_replay = isinstance(replay_memory, DeviceReplay)
        self._nstep = NStepAccumulator(config.n_step, config.reward_discount) if config.n_step > 1 else None
        self._prefill_replay_memory(config.replay_start_size)
        self._update_target_network()
        self.t_train0 = time.perf_counter()       # (after prefill: throughput meters' origin)

    # ------------------------------------------------------------ train loop
    def train(self, num_episodes, max_steps_per_episode, supervisor=None):
        """Reference `train` (`dqn_agent.py:52-70`): episodes until ``num_episodes`` or the
        supervisor says stop. The supervisor also sees every train step (periodic checkpoint,
        heartbeat, fault injection, stop agreement). Under synchronous data parallelism
        (``supervisor.coordinated``) a rank that runs out of episodes keeps training until
        the ranks agree to stop, and leaves mid-episode at the agreed step, so every rank
        takes the same number of collective SGD steps."""
        self._supervisor = supervisor
        coordinated = bool(getattr(supervisor, 'coordinated', False))
        episode = 0
        while True:
            if episode >= num_episodes:
                if not coordinated:
                    break
                supervisor.request_stop('num_episodes reached')
            reward, steps = self.train_episode(max_steps_per_episode)
            self.stats.log_episode(reward, steps)
            mean_reward = self.stats.last_100_mean_reward()
            log.info('Episode = %d, steps = %d, reward = %d, training steps = %d, '
                     'last-100 mean reward = %.2f' % (episode, steps, reward, self.training_steps, mean_reward))
            if self.monitor is not None:
                self.monitor.episode(episode, steps, reward)
            if self.metrics is not None:
                self.metrics.write(kind='episode', episode=episode, steps=steps, reward=reward,
                                   training_steps=self.training_steps, mean100=mean_reward,
                                   epsilon=self.random_action_prob,
                                   sgd_steps_per_sec=self.sgd_meter.rate(),
                                   env_frames_per_sec=self.frame_meter.rate(),
                                   replay_size=self.replay_memory.size())
            episode += 1
            if supervisor and supervisor.should_stop():
                log.warning('Received signal to stop. Exiting train loop.')
                break
            if self._train_budget_done():
                break

    def _begin_episode(self):
        self.frame_buffer.clear()
        observation = self.env.reset()
        frame = self.frame_buffer.append(observation)
        if self._device_replay:
            self.replay_memory.begin_episode(frame)
        if self._nstep is not None:
            self._nstep.reset()
        return self.frame_buffer.get_state()

    def _store(self, state, action, reward, next_state, done, next_frame):
        cfg = self.config
        if cfg.reward_clip > 0:
            reward = float(np.clip(reward, -cfg.reward_clip, cfg.reward_clip))
        if self._device_replay:
            if self._nstep is None:
                self.replay_memory.add_step(action, reward, next_frame, done,
                                            gamma_n=cfg.reward_discount)
            else:
                # n-step: states are frame-slot stacks tracked by the replay
                self._store_nstep_device(action, reward, next_frame, done)
        elif self._nstep is None:
            self.replay_memory.add(state, action, reward, next_state, done)
        else:
            # host replay keeps the reference 5-tuple; n-step returns use gamma^n
            # at train time (exact except for windows truncated by episode ends,
            # which are terminal and so do not bootstrap)
            for s, a, R, ns, d, _ in self._nstep.push(state, action, reward, next_state, done):
                self.replay_memory.add(s, a, R, ns, d)

    def _store_nstep_device(self, action, reward, next_frame, done):
        self.replay_memory.add_step_nstep(self._nstep, action, reward, next_frame, done)

    def train_episode(self, max_steps):
        state = self._begin_episode()
        total_reward = steps = 0
        done = False
        while not done and steps < max_steps:
            action = self._pick_action(state)
            observation, reward, done, _ = self.env.step(action)
            total_reward += reward
            steps += 1
            self.frame_meter.add(1)
            if done:
                reward = self.FAILURE_PENALTY.get(self.env.spec.id, reward)
            frame = self.frame_buffer.append(observation)
            next_state = self.frame_buffer.get_state()
            self._store(state, action, reward, next_state, done, frame)
            state = next_state
            if steps % self.config.update_freq == 0:
                self._train_minibatch(self.config.minibatch_size)
                if self._leave_episode():
                    break
        return total_reward, steps

    def _train_budget_done(self) -> bool:
        m = self.config.max_train_steps
        return bool(m) and self.training_steps >= m

    def _leave_episode(self) -> bool:
        """Leave mid-episode when the train-step budget is spent (every DP rank spends it at the
        same step) or when the coordinated stop was agreed at this step."""
        sv = self._supervisor
        if self._train_budget_done():
            return True
        return sv is not None and getattr(sv, 'coordinated', False) and sv.should_stop()

    # ---------------------------------------------------------- learner step
    def _train_minibatch(self, minibatch_size):
        if self._train_budget_done():
            return
        # device replay: staged (not yet flushed) transitions count, the flush below ships them
        avail = self.replay_memory.size() + (self.replay_memory.staged() if self._device_replay else 0)
        if avail < minibatch_size:
            return
        if self._device_replay:
            self.replay_memory.flush()
            loss = self.session.step()
        else:
            batch = self.replay_memory.sample_arrays(minibatch_size)
            dev = self.network.device
            tb = {k: torch.from_numpy(v).to(dev) for k, v in batch.items()}
            tb['gammas'] = torch.full_like(tb['rewards'], self.config.reward_discount ** self.config.n_step)
            loss, _ = self.network.train_step(tb)
        self.sgd_meter.add(1)
        if self._should_log_summary():
            # reference summary `loss` = TD loss + reg_param * L2 (network.py:149-155)
            self.network.last_loss = loss
            self.summary_writer.add_scalar('loss', self.network.total_loss(), self.training_steps)
        self.training_steps += 1
        if not self._device_replay:
            if self.config.target_update_tau < 1.0:
                self.network.update_target(self.config.target_update_tau)
            else:
                self._update_target_network()
        sv = self._supervisor
        if sv is not None:
            if getattr(self.session, 'stop_requested', False):    # e.g. the async PS said stop
                sv.request_stop('parameter server stopped')
            sv.on_train_step(self.training_steps)

    # ---------------------------------------------------------------- acting
    def _pick_action(self, state):
        if self._roll_random_action_dice():
            return self.env.action_space.sample()
        q_values = self._predict_q_values([state])
        return int(q_values.argmax())

    def _roll_random_action_dice(self):
        self._decay_random_action_prob()
        return self.rng.random() < self.random_action_prob

    def _decay_random_action_prob(self):
        if self.random_action_prob > self.config.min_random_action_prob:
            self.random_action_prob -= self.random_action_prob_decay

    def _predict_q_values(self, states, use_target_network=False):
        x = np.asarray(states)
        q = self.network.target_q_values(x) if use_target_network else self.network.q_values(x)
        return q.float().cpu().numpy()

    def _prefill_replay_memory(self, prefill_size):
        terminal = True
        state = None
        while self.replay_memory.size() < prefill_size:
            if terminal:
                state = self._begin_episode()
            action = self.env.action_space.sample()
            observation, reward, terminal, _ = self.env.step(action)
            frame = self.frame_buffer.append(observation)
            next_state = self.frame_buffer.get_state()
            self._store(state, action, reward, next_state, terminal, frame)
            state = next_state
            if self._device_replay and self.replay_memory.size() + self.replay_memory.staged() >= prefill_size:
                self.replay_memory.flush()
        if self._device_replay:
            self.replay_memory.flush()

    def _update_target_network(self):
        if self.training_steps % self.config.target_update_freq == 0:
            log.info('Updating target network')
            self.network.update_target(1.0)

    def _should_log_summary(self):
        if self.summary_writer is None:
            return False
        f = self.config.summary_freq
        return f > 0 and self.training_steps % f == 0

    # ---------------------------------------------------------------- helpers
    @classmethod
    def _get_frame_resizer(cls, env, config):
        w, h = config.resize_width, config.resize_height
        if w > 0 and h > 0:
            from .ops import preprocess
            return partial(preprocess.resize_image, width=w, height=h)
        return lambda x: x

    @classmethod
    def get_input_shape(cls, env, config):
        w, h = config.resize_width, config.resize_height
        if w > 0 and h > 0:
            return (w, h, config.frames_per_state)
        shape = tuple(env.observation_space.shape)
        if config.frames_per_state > 1:
            shape = shape + (config.frames_per_state,)
        return shape

    def agent_state(self):
        return {'random_action_prob': self.random_action_prob, 'training_steps': self.training_steps}

    def load_agent_state(self, state: Optional[dict]):
        """Apply an ``--save_agent_state`` sidecar (opt-in; the reference restarts epsilon and
        the local step count)."""
        if not state:
            return
        self.random_action_prob = float(state.get('random_action_prob', self.random_action_prob))
        self.training_steps = int(state.get('training_steps', self.training_steps))
