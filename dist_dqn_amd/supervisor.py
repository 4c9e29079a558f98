"""Run supervisor: the parts of ``tf.train.Supervisor`` the reference uses
(`/root/reference/src/main.py:136-143,155,167`, `/root/reference/src/dqn_agent.py:68-70`),
re-done for a torch.distributed job:

  * ``should_stop()`` / ``request_stop()`` — set by SIGINT/SIGTERM, by an
    exception in the managed block, by a fault-injection hook, or by a peer;
  * chief restore + broadcast of the WHOLE replica state to the other ranks
    (`prepare`; replaces the non-chief "wait for chief init, poll every
    recovery_wait_secs=3" loop), plus the restored path and agent sidecar;
  * periodic checkpoints (CheckpointManager, chief only) driven from the training
    loops through ``on_train_step`` and a final save on stop;
  * the step counter: ``global_step/sec`` written to the chief's TF event file every
    ``summary_secs`` (TF Supervisor default 120 s; reference `main.py:136-143`);
  * per-rank heartbeat files under ``<logdir>/heartbeat/`` so an external
    watchdog (or ``stale_ranks()``) can see dead/hung ranks;
  * fault injection for tests: ``DQN_FAULT_INJECT="step:N[,rank:R][,mode:raise|exit|stop]"``
    (``stop`` = a graceful stop request, ``raise`` = a crash of this rank's loop,
    ``exit`` = the process dies without cleanup).

Coordinated stop (``coordinated=True``: synchronous data parallelism). Every rank's SGD
step is a collective, so ranks must leave the loop after the SAME step or the survivors
block in the next gradient all-reduce. A local stop request (signal, ``stop`` fault, a
rank running out of episodes, a peer's stopping heartbeat) is therefore only recorded;
every ``stop_sync_steps`` train steps all ranks agree on it with one max-reduce on the
CPU control-plane group (gloo: no GPU sync), and ``should_stop()`` turns true on every
rank at the same step. A rank that crashes instead (``raise``/``exit``, a real fault) makes
the survivors' next collective fail (gloo: connection closed; RCCL: the process-group
timeout); the managed block then stops them WITHOUT a final save: the newest checkpoint is the
last periodic one, written from a state that passed the consistency check (``attach_learner``:
the in-graph xgmi transport reports a timed-out peer wait only through its error word, read
before every save, so no checkpoint is written from a partly reduced gradient).
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

from .checkpoint import CheckpointManager, load_sidecar

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
    if out['mode'] not in ('raise', 'exit', 'stop', 'actors'):
        raise ValueError('DQN_FAULT_INJECT mode must be raise, exit, stop or actors: %r' % spec)
    return out


class RunSupervisor:
    def __init__(self, is_chief: bool = True, logdir: str = '/tmp/train_logs', network=None,
                 rank: int = 0, world_size: int = 1, save_secs: int = 600, max_to_keep: int = 5,
                 heartbeat_secs: float = 5.0, install_signal_handlers: bool = True,
                 agent_state_fn=None, ctx=None, coordinated: bool = False, stop_sync_steps: int = 10,
                 summary_secs: float = 120.0):
        self.is_chief = is_chief
        self.logdir = logdir
        self.rank, self.world_size = rank, world_size
        self.ctx = ctx
        self.coordinated = bool(coordinated and ctx is not None and ctx.enabled)
        self.stop_sync_steps = max(1, int(stop_sync_steps))
        self._stop = threading.Event()          # agreed (coordinated) / effective stop
        self._local = threading.Event()         # this rank wants to stop
        self.stop_reason = ''
        self.ckpt = (CheckpointManager(logdir, network, is_chief, save_secs, max_to_keep, agent_state_fn)
                     if network is not None else None)
        self.fault = parse_fault_spec(os.environ.get('DQN_FAULT_INJECT'))
        self.fault_hooks = {}                   # mode -> callable (e.g. 'actors': kill the actor pool)
        self.hb_dir = os.path.join(logdir, 'heartbeat')
        self.heartbeat_secs = heartbeat_secs
        self._last_hb = 0.0
        self.last_step = 0
        self.restored_from: Optional[str] = None
        self.agent_state: Optional[dict] = None
        self.network = network
        self.summary_secs = float(summary_secs)
        self._sc_writer = None
        self._sc_last = None            # (time, global_step) of the last step-counter sample
        if install_signal_handlers and threading.current_thread() is threading.main_thread():
            for sig in (signal.SIGINT, signal.SIGTERM):
                try:
                    signal.signal(sig, self._on_signal)
                except (ValueError, OSError):
                    pass

    # ------------------------------------------------------------- stop flag
    def _on_signal(self, signum, frame):
        log.warning('Received signal %d: requesting stop', signum)
        self.request_stop('signal %d' % signum)

    def request_stop(self, reason: str = ''):
        """Ask to stop. Uncoordinated: effective now. Coordinated: effective on every rank at
        the next agreement step (``on_train_step``)."""
        if reason and not self._local.is_set():
            log.warning('Stop requested: %s', reason)
            self.stop_reason = reason
        self._local.set()
        if not self.coordinated:
            self._stop.set()
        self._write_hb(self.last_step, stopping=True)

    def _stop_now(self, reason: str):
        """Leave immediately on this rank (the loop is being torn down by an error)."""
        self.stop_reason = self.stop_reason or reason
        self._local.set()
        self._stop.set()
        self._write_hb(self.last_step, stopping=True)

    def should_stop(self) -> bool:
        return self._stop.is_set()

    def stop_requested(self) -> bool:
        """This rank asked to stop (possibly not yet agreed)."""
        return self._local.is_set()

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
            self._write_hb(step, stopping=self._local.is_set())
            if self.world_size > 1 and not self._local.is_set() and self.any_peer_stopping():
                self.request_stop('a peer rank is stopping')

    def any_peer_stopping(self) -> bool:
        for r in range(self.world_size):
            if r == self.rank:
                continue
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
        """Call after every learner step with the host step count (identical sequence on every
        sync-DP rank). Cheap: no GPU sync except when a checkpoint is actually written."""
        self.last_step = step
        f = self.fault
        if f and f['step'] is not None and step >= f['step'] and (f['rank'] is None or f['rank'] == self.rank):
            self.fault = None
            if f.get('mode') == 'exit':
                log.error('DQN_FAULT_INJECT: hard exit at step %d', step)
                os._exit(17)
            if f.get('mode') == 'stop':
                self.request_stop('DQN_FAULT_INJECT stop at step %d' % step)
            elif f.get('mode') == 'actors':
                # this rank's actor processes die (Ape-X); the trainer notices and asks to stop
                hook = self.fault_hooks.get('actors')
                log.error('DQN_FAULT_INJECT: killing this rank\'s actors at step %d%s', step,
                          '' if hook else ' (no actor pool registered: ignored)')
                if hook:
                    hook()
            else:
                raise FaultInjected('injected fault at step %d (rank %d)' % (step, self.rank))
        self.heartbeat(step)
        self._step_counter()
        if self.ckpt is not None:
            if self._local.is_set():
                # a stop is pending: the final forced save follows within a few steps -- store the
                # deferred optimizer slot (momentum-0 RMSProp `mom`, TF RMSProp_1) from now on, so
                # that save holds the last update's value like every periodic one
                self.ckpt.arm_slots()
            self.ckpt.maybe_save()
        if self.coordinated and step % self.stop_sync_steps == 0:
            if self.ctx.ctrl_allreduce_max(1 if self._local.is_set() else 0):
                if not self._stop.is_set():
                    log.warning('Stopping at train step %d (agreed across %d ranks)', step, self.world_size)
                self._stop.set()

    def _step_counter(self):
        """TF Supervisor's step-counter service: ``global_step/sec`` into the chief's event file
        (one device read of global_step per ``summary_secs``)."""
        if not self.is_chief or self.network is None or self.summary_secs <= 0:
            return
        now = time.time()
        if self._sc_last is None:
            self._sc_last = (now, int(self.network.global_step))
            return
        t, g = self._sc_last
        if now - t < self.summary_secs:
            return
        gs = int(self.network.global_step)
        if self._sc_writer is None:
            from .utils.metrics import SummaryWriter
            self._sc_writer = SummaryWriter(self.logdir)
        self._sc_writer.add_scalar('global_step/sec', (gs - g) / (now - t), gs)
        self._sc_last = (now, gs)

    # --------------------------------------------------------- managed run
    def prepare(self, broadcast_fn=None) -> Optional[str]:
        """Chief restores the latest checkpoint (if any); ``broadcast_fn`` then ships the whole
        replica state to every rank; every rank learns the restored path and agent sidecar."""
        # fresh heartbeat first: the broadcasts below are collectives, so once they return no
        # peer's heartbeat file is a stale 'stopping' left by a previous (crashed) run
        self._write_hb(0)
        if self.ckpt is not None and self.is_chief:
            self.restored_from = self.ckpt.restore()
            if self.restored_from:
                log.info('Restored from %s', self.restored_from)
                self.agent_state = load_sidecar(self.restored_from)
        if broadcast_fn is not None:
            broadcast_fn()
        if self.ctx is not None and self.ctx.enabled:
            self.restored_from, self.agent_state = self.ctx.ctrl_broadcast_object(
                (self.restored_from, self.agent_state))
        return self.restored_from

    def attach_learner(self, learner):
        """Checkpoint consistency check of this run: before every save the learner's in-graph
        error words (the xgmi all-reduce transport's, the fused optimizer's end-of-launch wait)
        must be clean; a failure is logged with the train step and the save is refused."""
        dev_checks = getattr(learner, '_device_checks', None)
        if self.ckpt is None or dev_checks is None:
            return

        def check():
            try:
                dev_checks()
            except Exception as e:
                log.error('rank %d: gradient all-reduce failed at or before train step %d (%r): not saving a '
                          'checkpoint from this state', self.rank, self.last_step, e)
                raise
        self.ckpt.check_fn = check

    @contextmanager
    def managed(self):
        failed = False
        try:
            yield self
        except FaultInjected:
            failed = True
            self._stop_now('fault injected')
            raise
        except Exception as e:
            failed = True
            self._stop_now('exception: %r' % (e,))
            log.error('rank %d: training loop failed (%r); stopping', self.rank, e)
            raise
        finally:
            self.stop(failed=failed)

    def stop(self, failed: bool = False):
        """Final save on a graceful stop (not after a failure: the state may be inconsistent, the
        last periodic checkpoint stays the newest)."""
        if self.ckpt is not None and self.is_chief:
            try:
                if failed:
                    self.ckpt.wait()
                    log.warning('rank %d: no final checkpoint after a failure; newest is %s', self.rank,
                                self.ckpt.last_path)
                else:
                    self.ckpt.maybe_save(force=True)
            except Exception as e:  # pragma: no cover
                log.error('final checkpoint failed: %r', e)
        self._write_hb(self.last_step, stopping=True)
