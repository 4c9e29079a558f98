"""Run supervisor: the parts of ``tf.train.Supervisor`` the reference uses
(`/root/reference/src/main.py:136-143,155,167`, `/root/reference/src/dqn_agent.py:68-70`),
re-done for a torch.distributed job:

  * ``should_stop()`` / ``request_stop()`` — set by SIGINT/SIGTERM, by an
    exception in the managed block, by a fault-injection hook, or by a peer's
    stop (polled through a per-rank heartbeat file);
  * chief init/restore + broadcast to the other ranks (replaces the non-chief
    "wait for chief init, poll every recovery_wait_secs=3" loop);
  * periodic checkpoints (CheckpointManager) and a final save on stop;
  * per-rank heartbeat files under ``<logdir>/heartbeat/`` so an external
    watchdog (or ``stale_ranks()``) can see dead/hung ranks;
  * fault injection for tests: ``DQN_FAULT_INJECT="step:N[,rank:R][,mode:raise|exit]"``.
"""
from __future__ import annotations

import json
import logging
import os
import signal
import threading
import time
from contextlib import contextmanager
from typing import List, Optional

from .checkpoint import CheckpointManager

log = logging.getLogger(__name__)


class FaultInjected(RuntimeError):
    pass


def parse_fault_spec(spec: Optional[str]):
    if not spec:
        return None
    out = {'step': None, 'rank': None, 'mode': 'raise'}
    for part in spec.split(','):
        k, _, v = part.partition(':')
        out[k.strip()] = v.strip() if k.strip() == 'mode' else int(v)
    return out


class RunSupervisor:
    def __init__(self, is_chief: bool = True, logdir: str = '/tmp/train_logs', network=None,
                 rank: int = 0, world_size: int = 1, save_secs: int = 600, max_to_keep: int = 5,
                 heartbeat_secs: float = 5.0, install_signal_handlers: bool = True,
                 agent_state_fn=None):
        self.is_chief = is_chief
        self.logdir = logdir
        self.rank, self.world_size = rank, world_size
        self._stop = threading.Event()
        self.ckpt = (CheckpointManager(logdir, network, is_chief, save_secs, max_to_keep, agent_state_fn)
                     if network is not None else None)
        self.fault = parse_fault_spec(os.environ.get('DQN_FAULT_INJECT'))
        self.hb_dir = os.path.join(logdir, 'heartbeat')
        self.heartbeat_secs = heartbeat_secs
        self._last_hb = 0.0
        self.restored_from: Optional[str] = None
        if install_signal_handlers and threading.current_thread() is threading.main_thread():
            for sig in (signal.SIGINT, signal.SIGTERM):
                try:
                    signal.signal(sig, self._on_signal)
                except (ValueError, OSError):
                    pass

    # ------------------------------------------------------------- stop flag
    def _on_signal(self, signum, frame):
        log.warning('Received signal %d: requesting stop', signum)
        self.request_stop()

    def request_stop(self, reason: str = ''):
        if reason:
            log.warning('Stop requested: %s', reason)
        self._stop.set()
        self._write_hb(stopping=True)

    def should_stop(self) -> bool:
        return self._stop.is_set()

    # ------------------------------------------------------------ heartbeat
    def _write_hb(self, step: int = -1, stopping: bool = False):
        try:
            os.makedirs(self.hb_dir, exist_ok=True)
            tmp = os.path.join(self.hb_dir, 'rank%d.json.tmp' % self.rank)
            with open(tmp, 'w') as f:
                json.dump({'rank': self.rank, 'time': time.time(), 'step': step, 'stopping': stopping,
                           'pid': os.getpid()}, f)
            os.replace(tmp, os.path.join(self.hb_dir, 'rank%d.json' % self.rank))
        except OSError:
            pass

    def heartbeat(self, step: int):
        now = time.time()
        if now - self._last_hb >= self.heartbeat_secs:
            self._last_hb = now
            self._write_hb(step)
            if self.world_size > 1 and self.any_peer_stopping():
                self._stop.set()

    def any_peer_stopping(self) -> bool:
        for r in range(self.world_size):
            p = os.path.join(self.hb_dir, 'rank%d.json' % r)
            try:
                with open(p) as f:
                    if json.load(f).get('stopping'):
                        return True
            except (OSError, ValueError):
                continue
        return False

    def stale_ranks(self, timeout_s: float = 60.0) -> List[int]:
        now, out = time.time(), []
        for r in range(self.world_size):
            p = os.path.join(self.hb_dir, 'rank%d.json' % r)
            try:
                with open(p) as f:
                    if now - json.load(f)['time'] > timeout_s:
                        out.append(r)
            except (OSError, ValueError, KeyError):
                out.append(r)
        return out

    # ------------------------------------------------------------ per step
    def on_train_step(self, step: int):
        f = self.fault
        if f and f['step'] is not None and step >= f['step'] and (f['rank'] is None or f['rank'] == self.rank):
            self.fault = None
            if f.get('mode') == 'exit':
                log.error('DQN_FAULT_INJECT: hard exit at step %d', step)
                os._exit(17)
            raise FaultInjected('injected fault at step %d (rank %d)' % (step, self.rank))
        self.heartbeat(step)
        if self.ckpt is not None:
            self.ckpt.maybe_save()

    # --------------------------------------------------------- managed run
    def prepare(self, broadcast_fn=None) -> Optional[str]:
        """Chief restores the latest checkpoint (if any); params are then broadcast."""
        if self.ckpt is not None and self.is_chief:
            self.restored_from = self.ckpt.restore()
            if self.restored_from:
                log.info('Restored from %s', self.restored_from)
        if broadcast_fn is not None:
            broadcast_fn()
        self._write_hb(0)
        return self.restored_from

    @contextmanager
    def managed(self):
        try:
            yield self
        except FaultInjected:
            self.request_stop('fault injected')
            raise
        except Exception as e:
            self.request_stop('exception: %r' % (e,))
            raise
        finally:
            self.stop()

    def stop(self):
        if self.ckpt is not None and self.is_chief:
            try:
                self.ckpt.maybe_save(force=True)
            except Exception as e:  # pragma: no cover
                log.error('final checkpoint failed: %r', e)
        self._write_hb(stopping=True)
